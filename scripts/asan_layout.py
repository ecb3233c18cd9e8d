"""Driver of scripts/asan_layout.sh: config P's staged layout through an ASan build of
dg_staged_order (layout.cpp)."""
import ctypes, sys, numpy as np
sys.path.insert(0, str(__import__('pathlib').Path(__file__).resolve().parents[1]))
lib = ctypes.CDLL(sys.argv[1])
from decagon_amd import synthetic, engine
from decagon_amd.sparse import staged_layout
from decagon_amd.sharding import RelationShard
def order(csr, perm):
    rowptr = np.ascontiguousarray(csr.rowptr, np.int32); col = np.ascontiguousarray(csr.col, np.int32)
    perm = np.ascontiguousarray(perm, np.int32); rank = np.zeros(len(col), np.int32)
    rc = lib.dg_staged_order(ctypes.c_void_p(rowptr.ctypes.data), ctypes.c_void_p(col.ctypes.data), ctypes.c_int32(len(rowptr)-1), ctypes.c_void_p(perm.ctypes.data), ctypes.c_void_p(rank.ctypes.data))
    assert rc == 0, rc
    return rank
g = synthetic.make_P(0)
csr = g.csr()
for world, rank in ((8, 0), (1, 0)):
    sh = RelationShard.polypharmacy(g, rank, world, comm=False)
    loc = [csr[(1,1)][k] for k in sh.local[(1,1)]]
    out_chunk = max(1, -(-len(loc) // engine.STAGED_BINS))
    perm = engine.snake_bins([c.nnz for c in loc], out_chunk)
    loc = [loc[i] for i in perm]
    lay = staged_layout(loc, order, split=True)
    print(world, rank, len(loc), lay.jm_len, flush=True)
