# (Adopted in round 6: the tab kernels' layer 2 uses the DPP hand-out)
EDITS = []
