# A/B (config P's protein rows, spmm_groups_kernel): the streamed (vcol, val) pairs read with
# non-temporal loads, so the CSR stream (8 B a nonzero, read once) does not push the window's
# gathered operand rows out of the XCD's L2.
EDITS = [("spmm.hip", """    if (base + lane < end) {
        vc = g.vcol[base + lane];
        vv = g.val[base + lane];""", """    if (base + lane < end) {
        vc = __builtin_nontemporal_load(g.vcol + base + lane);
        vv = __builtin_nontemporal_load(g.val + base + lane);"""),
         ("spmm.hip", """        if (nb + lane < end) {
            vc = vcolp[nb + lane];
            vv = valp[nb + lane];""", """        if (nb + lane < end) {
            vc = __builtin_nontemporal_load(vcolp + nb + lane);
            vv = __builtin_nontemporal_load(valp + nb + lane);""")]
