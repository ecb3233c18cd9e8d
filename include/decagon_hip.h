/*
 * decagon_hip.h — C ABI of libdecagon_hip.so, the MI355X (gfx950) kernels behind the
 * Decagon multi-relational GCN forward and its edge decoders.
 *
 * The reference (jrectorb/decagon, TF 1.8) has no FFI: its "boundary" is a set of TF ops
 * called from the decagon/deep modules.  Every entry point below replaces one or a fused run of
 * those ops; the replaced call sites are cited per function (paths relative to the
 * reference root).  The Python layer in decagon_amd/ binds these with ctypes
 * (decagon_amd/_lib.py); INTEGRATION.md shows the binding.
 *
 * Conventions (all entry points):
 *   - every pointer argument is a caller-owned DEVICE pointer unless documented as host;
 *     the library never allocates or frees caller memory; the only state it keeps between
 *     calls is, per kernel that opts into more than 64 KB of dynamic LDS, the set of devices
 *     on which that (idempotent) hipFuncSetAttribute has been applied — thread-safe;
 *   - launches are asynchronous on `stream` (a hipStream_t passed as void*; NULL = the
 *     null stream) and are safe to capture into a hipGraph;
 *   - the return value is DG_OK (0), a negative DG_E* code for an argument error detected
 *     on the host before any launch, or a positive hipError_t from the launch.
 *   - float arithmetic is IEEE fp32 (no fast-math); sums are in a fixed order, so results
 *     are bitwise reproducible run to run (no float atomics anywhere).
 */
#ifndef DECAGON_HIP_H
#define DECAGON_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DG_OK 0
#define DG_EINVAL (-1)     /* bad size / null pointer / unsupported shape            */
#define DG_EALIGN (-2)     /* a dense operand is not 16-byte aligned row by row      */
#define DG_ETOOMANY (-3)   /* more groups than DG_MAX_GROUPS in one launch           */

#define DG_MAX_GROUPS 8

/* ABI version (36); bumped whenever a struct layout or a signature changes (36: DG_PEER_STATE_WORDS grew). */
int32_t dg_abi_version(void);

/* --------------------------------------------------------------------------------------
 * Relation-group SpMM (T3 + T4 of SURVEY §2.2) over a chunk-merged CSR.
 *
 * A group's relations A_k (k < K, all n_rows x n_cols) are split into chunks of consecutive
 * relations; for chunk c and row r the nonzeros of every relation in the chunk are stored
 * contiguously, [rowptr[c*n_rows + r], rowptr[c*n_rows + r + 1]), each with a virtual
 * column vcol = k*n_cols + col — the row of the relation-stacked dense operand
 * X = [X_0; X_1; ...] (row v at x + v*x_ld) that it multiplies.  Then
 *
 *     out[c][r][:] = sum_{p in range(c, r)} val[p] * X[vcol[p]][:]
 *                  = sum_{k in chunk c} (A_k · X_k)[r][:]
 *
 * With one chunk this is the add_n of layers.py:92/116.  The layout is built once at upload
 * (decagon_amd/sparse.py: merge_chunks).
 * Replaces: tf.sparse_tensor_dense_matmul(adj_mats[edge_type][k], x)  layers.py:90, :114
 *           tf.sparse_tensor_dense_matmul(x, weights_k) (sparse features) layers.py:89
 *           tf.add_n(outputs)                                         layers.py:92, :116
 * Requirements: d % 4 == 0, 4 <= d <= 256, x and x_ld 16-byte aligned (x_ld % 4 == 0),
 * x_rows * x_ld < 2^31 (gathers use 32-bit offsets), 0 <= vcol < x_rows.
 * -------------------------------------------------------------------------------------- */
typedef struct dg_rel_group {
    const int32_t* rowptr;      /* device, [n_chunks*n_rows + 1]                          */
    const int32_t* vcol;        /* device, [nnz] virtual columns (rows of X)              */
    const float* val;           /* device, [nnz].  vcol/val may be NULL when nnz == 0.    */
    const float* x;             /* device, relation-stacked dense operand                 */
    float* out;                 /* device, [n_chunks][n_rows][d] (unused in fused mode)   */
    int64_t x_ld;               /* elements between consecutive rows of X                 */
    int32_t n_rows;
    int32_t n_chunks;
    int32_t x_rows;             /* rows of X addressable (bound on vcol); per chunk when  */
                                /* DG_GROUP_SHARED_PATTERN is set                         */
    int32_t flags;              /* 0, or DG_GROUP_SHARED_PATTERN [| DG_GROUP_DROPOUT]      */
                                /* (dg_spmm_groups_f32 only), or DG_GROUP_DENSE_ROWS       */
                                /* (dg_gcn_fused_f32 only)                                */
    uint32_t drop_tag;          /* DG_GROUP_DROPOUT: mask stream of the group             */
    float drop_keep;            /* DG_GROUP_DROPOUT: keep probability in (0, 1]           */
    int32_t drop_stride;        /* DG_GROUP_DROPOUT: mask elements per chunk (the nnz of  */
                                /* the pattern)                                           */
    const uint64_t* drop_state; /* DG_GROUP_DROPOUT: device {seed, step}, else NULL       */
    const int32_t* drop_index;  /* DG_GROUP_DROPOUT: device [nnz] mask element of each    */
                                /* nonzero, or NULL (its position)                        */
} dg_rel_group;

/* Every chunk c uses the same CSR pattern (rowptr[0..n_rows], vcol, val) over its own slab of
 * X: rows [c*x_rows, (c+1)*x_rows).  The relation-batched X_j·W_k of sparse features
 * (layers.py:89, one X_j for every relation k) and its backward X_jᵀ·G_k, without K copies
 * of the pattern. */
#define DG_GROUP_SHARED_PATTERN 1

/* With DG_GROUP_SHARED_PATTERN: chunk c multiplies nonzero p's value by the dropout scale of
 * mask element c*drop_stride + (drop_index ? drop_index[p] : p) of stream drop_tag (dropout.h:
 * kept with probability drop_keep, scaled by 1/drop_keep) — dropout_sparse on the features
 * of every relation (layers.py:23-31, :88), each relation its own draw, the backward X_jᵀ·G_k
 * (drop_index: the transposed pattern's nonzeros mapped to the forward's) on the same masks. */
#define DG_GROUP_DROPOUT 2

/* dg_gcn_fused_f32 only: the group has no adjacency — row r of its sum IS row r of X
 * (x[r * x_ld ..], x_rows >= n_rows; rowptr / vcol / val unused, may be NULL), or with
 * n_chunks = S > 1 (S <= DG_PEER_MAX) the sum of S slots of such rows, slot c at
 * x + c*x_rows*x_ld, added in slot order (fp32, deterministic).  The sharded forward finishes
 * its all-reduced pre-normalisation sums S_ij this way (layers.py:92-93 after the cross-rank
 * Σ_k), without an identity CSR's two dependent loads; with the peer exchange the slots are
 * the ranks' partial sums, so the all-reduce's addition happens here. */
#define DG_GROUP_DENSE_ROWS 4

int dg_spmm_groups_f32(const dg_rel_group* groups /* HOST array */, int32_t n_groups,
                       int32_t d, void* stream);

/* The same partial-mode product (out[c][r][:] = Σ val·X[vcol][:]) for groups whose whole
 * dense operand is small — x_rows <= 1137 rows (it is staged in LDS, 144 B per row per
 * 32-column slice): the backward's Âᵀ·dS_ij, where every relation of the group reads the
 * same dS_ij (decagon_amd/train.py).  out must be 16-byte aligned; other requirements as
 * dg_spmm_groups_f32.  Replaces the gradient of tf.sparse_tensor_dense_matmul w.r.t. its
 * dense operand (layers.py:90, :114). */
int dg_spmm_groups_lds_f32(const dg_rel_group* groups /* HOST array */, int32_t n_groups, int32_t d,
                           void* stream);

/* Single relation, plain CSR: Y[r][:] = sum_p val[p] * X[col[p]][:] + beta * Y[r][:]
 * (Y dense, ld = ldy; fmaf(beta, Y, sum) per element).  beta == 0 writes Y without reading it
 * (no NaN carried over from uninitialised memory); beta == 1 accumulates one relation's product
 * into a running sum — tf.add_n over the per-relation products (layers.py:92, :116) done one
 * relation at a time.  Replaces one tf.sparse_tensor_dense_matmul (layers.py:90, :114).  ldy
 * must equal d; beta must be finite (ABI 37: beta added). */
int dg_spmm_csr_f32(const int32_t* rowptr, const int32_t* col, const float* val,
                    int32_t n_rows, int32_t n_cols, const float* x, int64_t ldx, float* y,
                    int64_t ldy, int32_t d, float beta, void* stream);

/* Row-wise L2 normalisation, stand-alone (ABI 37):
 *     y[r] = x[r] * rsqrt(max(sum_c x[r][c]^2, 1e-12))          (tf.nn.l2_normalize(x, dim=1))
 * then relu if flags == DG_EPI_RELU (model.py:75).  x, y: [n_rows][d], contiguous, 16-byte
 * aligned; y == x is allowed (each row is read whole before it is written).  Replaces
 * layers.py:93 / :117 when the sum was formed elsewhere (dg_spmm_csr_f32 with beta = 1); the
 * layer kernels fuse the same arithmetic into their epilogues (dg_gcn_epilogue_f32 with one
 * group of one chunk runs it: bitwise the same rows). */
int dg_rownorm_l2_f32(const float* x, float* y, int32_t n_rows, int32_t d, int32_t flags, void* stream);

/* --------------------------------------------------------------------------------------
 * Fused GCN layer (T3 + T4 + T5 + T6, optionally T7 of the next layer, in one launch) for
 * node types whose groups each fit one chunk: for every target t (a node type i), r < n_rows,
 *
 *     out_t[r] = act( sum_{g in [g_begin, g_begin+g_count)} l2norm( sum_k A_g,k[r]·X_g,k ) )
 *
 * act = relu if flags & DG_EPI_RELU.  Every group must have n_chunks == 1; `out` is ignored.
 * One workgroup per output row, `waves_per_group` waves per group sharing the row's nonzeros
 * (g_count * waves_per_group <= 16).
 * Projection epilogue: for each dg_proj p with p.target == t,
 *     p.out[rel(kk)][r][c] = sum_k out_t[r][k] * p.w[rel(kk)][k][c]   kk < p.n_rels, c < d_out
 * (rel(kk) = p.rel_map[kk] or kk; p.w is a [K][d][d_out] stack, p.out [K][n_rows][d_out])
 * — the next layer's H_j·W_k (layers.py:113) for the rows just produced.
 * Replaces the per-relation SpMM + add_n + l2_normalize of layers.py:85-94 / 109-118 and the
 * sum over edge types (+ relu) of model.py:74-75 / 85-88.
 * -------------------------------------------------------------------------------------- */
typedef struct dg_fused_target {
    float* out;                 /* device, [n_rows][d] */
    int32_t n_rows;
    int32_t g_begin;
    int32_t g_count;
    int32_t flags;              /* 0 or DG_EPI_RELU */
} dg_fused_target;

typedef struct dg_proj {
    const float* w;             /* device, [K][d][d_out] weight stack        */
    const int32_t* rel_map;     /* device, [n_rels] or NULL                  */
    float* out;                 /* device, [K][n_rows of target][d_out]      */
    int32_t n_rels;
    int32_t target;             /* index into the targets array              */
    int32_t d_out;
    int32_t reserved;
} dg_proj;

int dg_gcn_fused_f32(const dg_rel_group* groups /* HOST */, int32_t n_groups,
                     const dg_fused_target* targets /* HOST */, int32_t n_targets,
                     const dg_proj* projs /* HOST, may be NULL */, int32_t n_projs,
                     int32_t waves_per_group, int32_t d, void* stream);

/* --------------------------------------------------------------------------------------
 * Relation-segment SpMM (partial mode; one wave per (row, relation)), optionally with the
 * next layer's projection reassociated into it — the sharded config-S form (one relation set
 * per GPU, every node type row-split), where a rank's short row block would leave
 * most CUs idle at one workgroup per row.  Over dg_rel_group's chunk-merged CSR with `chunk`
 * relations per chunk (relation k = c*chunk + t), for every chunk c and row r:
 *
 *   w == NULL:  out[c][r][:]  = sum_{t} sum_{p in seg(c,r,t)} val[p] * X[vcol[p]][:]
 *   w != NULL:  out[c][r][:]  = sum_{t} ( sum_{p in seg(c,r,t)} val[p] * H[vcol[p] - s*n_cols][:] ) · W[s]
 *               (s = slab[k] or k; H = x, [n_cols][x_ld]; W a [K][64][32] stack)
 *
 * The second form is layer 2 as sum_k (A_k·H1_j)·W2_k instead of sum_k A_k·(H1_j·W2_k)
 * (layers.py:113-114): the shared H1_j is gathered and only this rank's rows are projected.
 * seg[(c*n_rows + r)*chunk + t] is the first nonzero of relation t of chunk c in row r inside
 * [rowptr[c*n_rows + r], rowptr[c*n_rows + r + 1]); a segment ends where the next one starts
 * (the last one at the range's end).  Relations run in t order within a range (merge_chunks).
 * Requirements: 1 <= chunk <= 16, (n_chunks - 1)*chunk < n_rels <= n_chunks*chunk;
 * w == NULL: d_in == d_out in {32, 64}; w != NULL (every group): d_in == 64, d_out == 32;
 * x, out, w and x_ld 16-byte aligned; x_rows * x_ld < 2^31 with 0 <= vcol < x_rows.
 * Replaces: tf.sparse_tensor_dense_matmul + tf.add_n (layers.py:90-92, :114-116) over a
 * chunk's relations, and tf.matmul(x, weights_k) (layers.py:113).
 * -------------------------------------------------------------------------------------- */
typedef struct dg_seg_group {
    const int32_t* rowptr;      /* device, [n_chunks*n_rows + 1]                          */
    const int32_t* seg;         /* device, [n_chunks*n_rows*chunk] segment starts         */
    const int32_t* vcol;        /* device, [nnz]                                          */
    const float* val;           /* device, [nnz]                                          */
    const int32_t* slab;        /* device, [n_rels] slab of local relation k, or NULL     */
    const float* x;             /* device: stacked X (w == NULL) or H [n_cols][x_ld]      */
    const float* w;             /* device, [K][64][32] weight stack, or NULL              */
    float* out;                 /* device, [n_chunks][n_rows][d_out]                      */
    int64_t x_ld;
    int32_t n_rows;
    int32_t n_cols;
    int32_t n_chunks;
    int32_t chunk;
    int32_t n_rels;
    int32_t x_rows;             /* bound on vcol (K*n_cols for the stacked forms)         */
} dg_seg_group;

int dg_spmm_seg_f32(const dg_seg_group* groups /* HOST array */, int32_t n_groups, int32_t d_in,
                    int32_t d_out, void* stream);

/* The fused form: a whole layer for the target node types, every output row finished in one
 * workgroup.  Groups are chunk-merged as for dg_spmm_seg_f32 (any n_chunks; n_rels >= 1).
 * For every target t (dg_fused_target: out [n_rows][d_out], groups [g_begin, g_begin + g_count),
 * flags 0 or DG_EPI_RELU; groups[i].out unused) and row r < n_rows:
 *
 *   out_t[r] = act( sum_g l2norm( sum_{t < n_rels_g} seg-sum_g(r, t) ) )
 *
 * with seg-sum as dg_spmm_seg_f32's over relation t = c*chunk + t' of the group (projected by
 * W[slab] when the groups carry w), at most 16 relations a target row in total.  One
 * workgroup per row, one wave per (group, relation); relations and groups summed in order.
 * With w this is layer 2 (layers.py:109-118) reassociated, Σ_k (Â_k·H1_j)·W2_k, so layer 1
 * needs no projection of its rows.  Replaces layers.py:85-94 / 109-118 and model.py:74-75,
 * 85-88 for such node types. */
int dg_gcn_fused_seg_f32(const dg_seg_group* groups /* HOST */, int32_t n_groups,
                         const dg_fused_target* targets /* HOST */, int32_t n_targets, int32_t d_in,
                         int32_t d_out, void* stream);

/* The wave-table form of dg_gcn_fused_seg_f32 (round 5): the same launch — workgroups, waves,
 * arithmetic and summation order, so bitwise the same rows — with everything a wave needs
 * before its gathers precomputed on the host (decagon_amd/sparse.py: wave_table) instead of
 * found at run time from the group and target arguments.  Wave w of workgroup b (slot
 * i = b * nw_stride + w) reads desc[i] and the first batch of its relation segment's pairs,
 * pairs[64 i .. 64 i + 63] (vcol, fp32 value bits: int32 pairs), in one round trip; a segment
 * longer than 64 continues in ovf[desc[i].ovf ..] in batches of 64.  Within a batch, pair
 * m of a d_in = 64, d_out = 64 table sits in entry 16 (m & 3) + (m >> 2) (the DPP hand-out
 * order of the seg form), of a d_in = 64, d_out = 32 table (layer 2 reassociated) in entry m.
 * A wave with cnt 0 gathers nothing; desc.role (active << 31 | nbuf slot << 16 | K << 8 | first
 * wave) makes it the wave that sums and L2-normalises one (row slot, group); desc.orow != NULL
 * makes it the writer of that output row (wr = group count | relu << 8 | row slot << 16).
 * Shapes: d_in = d_out = 64, or d_in = 64, d_out = 32 with W slabs (desc.w).  Replaces
 * layers.py:85-94 / 109-118 and model.py:74-75, 85-88 as dg_gcn_fused_seg_f32 does. */
typedef struct dg_tab_desc {
    const float* x;       /* device: gather base (vcol * x_ld floats from here)             */
    const float* w;       /* device: the relation's W slab [64][32] (d_out 32), or NULL      */
    float* orow;          /* device: the output row this wave writes, or NULL               */
    int32_t cnt;          /* pairs of the wave's segment (0: none)                          */
    int32_t x_ld;         /* floats                                                          */
    int32_t ovf;          /* first entry of the later batches in ovf                         */
    uint32_t role;
    uint32_t wr;
    int32_t pad[5];
} dg_tab_desc;            /* 64 bytes                                                        */

typedef struct dg_wave_table {
    const int32_t* pairs; /* device, [n_blocks * nw_stride * slot_pairs][2], 16-byte aligned */
    const int32_t* ovf;   /* device, [..][2], or NULL                                        */
    const dg_tab_desc* desc; /* device, [n_blocks * nw_stride], 64-byte aligned             */
    int32_t n_blocks;
    int32_t nw;           /* waves per workgroup, 1..16                                      */
    int32_t nw_stride;    /* 8 if nw <= 8, else 16                                           */
    int32_t slot_pairs;   /* S: pairs of a wave's first batch, 16 / 32 / 48 / 64 (ABI 37;     */
                          /* 0 means 64): pair m < S of the segment at slot entry             */
                          /* (m & 3)·S/4 + (m >> 2); pairs S, S+1, ... in batches of 64 from  */
                          /* ovf + desc.ovf, pair j of a batch at entry 16·(j & 3) + (j >> 2) */
} dg_wave_table;

int dg_gcn_fused_tab_f32(const dg_wave_table* table /* HOST */, int32_t d_in, int32_t d_out, void* stream);

/* dg_gcn_fused_tab_f32 with the peer-store exchange (config S at N = 2 with --exchange peer):
 * every finished row also goes to every peer's copy of its target — desc.pad[0] = the row's
 * byte offset in its target, desc.pad[1] = the target's bytes, the target inside the exchange
 * region — and the launch ends with the exchange, as dg_gcn_fused_seg_peer_f32.  xchg as
 * dg_peer_allgather; at least one workgroup. */
struct dg_peer_xchg;
int dg_gcn_fused_tab_peer_f32(const dg_wave_table* table /* HOST */, int32_t d_in, int32_t d_out,
                              const struct dg_peer_xchg* xchg /* HOST */, void* stream);

/* The wave-table form of dg_spmm_seg_f32 (partial mode; config S's N-GPU layers): the same
 * workgroups (in that entry point's XCD-contiguous item order), waves and chunk partials, bit
 * for bit, from a host-built table with the layout above.  A wave whose desc.orow != NULL is
 * the first wave of its (chunk, row): after the barrier it adds the (desc.role >> 8) & 0xff
 * waves from itself on, in order, and stores the partial row there.  Shapes as above. */
int dg_spmm_seg_tab_f32(const dg_wave_table* table /* HOST */, int32_t d_in, int32_t d_out, void* stream);

/* --------------------------------------------------------------------------------------
 * LDS-staged relation SpMM for groups of many relations over a narrow column space
 * (polypharmacy drug x drug: 1,928 relations of 645 x 645).  For output chunk c (out_chunk
 * consecutive relations):
 *
 *     out[c][r][:] = sum_{k in chunk c} sum_{p in row r of A_k} val[p] * X[slab(k)*n_cols + col[p]][:]
 *
 * Layout (built on the host by decagon_amd/sparse.py: staged_layout): per relation, a long
 * row becomes a group of <= 8 equal-length segments (virtual rows; padding pairs read one
 * of sixteen zero columns n_cols .. n_cols + 15, value 0), at most 1024 virtual rows (16 waves of 64 lanes) sorted by length
 * with each group inside one wave; wave w's pairs form a dense block [rlw_w][64] (rlw_w a
 * multiple of 4; holes are padding pairs), lane j's pair at diagonal m at woff_w + 64 m + j:
 *   pairs      [n_pairs][2] int32: (column, fp32 value bits), relations and waves back to
 *              back; 16-byte aligned
 *   jm, jmoff  relation k's tables at jm[jmoff[k] .. jmoff[k+1]): [n_waves, largest group,
 *              0, 0], woff[16], rlw[16] (0 past n_waves), vinfo[64 n_waves] = row |
 *              segment << 10 | (group size - 1) << 13 | length << 16 (row 1023: padding
 *              lane); jm ends with 1024 spare ints (jm_len >= jmoff[n_rels] + 1024)
 * One workgroup of 1024 threads per (c, 16-float column slice); thread i owns sorted virtual
 * row i and streams its pairs from global memory (one coalesced load per wave and diagonal);
 * the slab slice is in LDS and every nonzero gathers from it; the segments of a row are
 * summed in segment order.  Requirements: n_rows < 1023; n_cols <= 1024; out_chunk <= 64;
 * d % 4 == 0; x, x_ld 16-byte aligned.
 * Replaces layers.py:90-92 / :114-116 for such groups.
 * -------------------------------------------------------------------------------------- */
typedef struct dg_staged_group {
    const int32_t* pairs;       /* device, [n_pairs][2]                                  */
    const int32_t* jm;          /* device                                                */
    const int32_t* jmoff;       /* device, [n_rels + 1]                                  */
    const int32_t* slab;        /* device, [n_rels] slab of relation k, or NULL (= k)    */
    const float* x;             /* device, relation-stacked dense operand                */
    float* out;                 /* device, [ceil(n_rels/out_chunk)][n_rows][d]           */
    int64_t x_ld;
    int32_t n_rows;
    int32_t n_cols;
    int32_t n_rels;
    int32_t out_chunk;          /* relations summed into one output chunk (<= 64)        */
    int32_t x_rows;             /* rows of x addressable                                 */
    int32_t jm_len;             /* ints in jm, including the 1024 spare                  */
    /* Variable output chunks (or NULL: chunk c = relations [c·out_chunk, (c+1)·out_chunk)):
     * HOST [n_chunks + 1], chunk c = relations [chunk_start[c], chunk_start[c+1]); starts at 0,
     * ends at n_rels (<= 65535), 1..64 relations a chunk, n_chunks <= DG_STAGED_MAX_CHUNKS.
     * out is then [n_chunks][n_rows][d].  Copied into the launch's arguments. */
    const int32_t* chunk_start;
    int32_t n_chunks;
    int32_t pad;
} dg_staged_group;
#define DG_STAGED_MAX_CHUNKS 128

int dg_spmm_staged_f32(const dg_staged_group* groups /* HOST */, int32_t n_groups, int32_t d,
                       void* stream);

/* The same SpMM with each relation's dense operand made in the workgroup instead of read:
 *     X_k = H · W[slab(k)]        (H [n_cols][64] row-major, leading dimension h_ld; W [K][64][d])
 * — layer 2's projection H1_j · W2_k (layers.py:113) fused into its SpMM (layers.py:114): the
 * slab slice comes from the fp32 MFMA (exact fp32 products, k summed in a fixed order) into
 * LDS, so the [K][n_cols][d] operand is never written to or read from HBM.  groups[i].x /
 * x_ld / x_rows are ignored.  Requirements as dg_spmm_staged_f32, plus din == 64, h and h_ld
 * 16-byte aligned.  Replaces layers.py:113-116 for such groups. */
typedef struct dg_staged_proj {
    const float* h;             /* device, [n_cols][h_ld]                                 */
    const float* w;             /* device, [K][din][d]                                     */
    int64_t h_ld;
    int32_t din;                /* 64                                                      */
    int32_t pad;
} dg_staged_proj;

int dg_spmm_staged_proj_f32(const dg_staged_group* groups /* HOST */, const dg_staged_proj* projs /* HOST */,
                            int32_t n_groups, int32_t d, void* stream);


/* Host-only layout helper: one relation's pair block of the staged layout.  Its lanes
 * (virtual rows; n_lanes = 64 x waves) are given as a CSR over lanes (HOST arrays: lrowptr
 * [n_lanes + 1], lcol / lval the lanes' nonzeros in any order), rlw[wave] the wave's diagonals
 * (>= its longest lane).  Fills pairs [sum rlw x 64][2] (wave w's block after the blocks of
 * waves < w; lane j's pair at diagonal m at 64 m + j: (column, fp32 value bits); holes
 * (n_cols + z, 0) with z < 16).  The diagonal of each nonzero and the zero column of each
 * hole are chosen so that the lanes of each ds_read_b128 lane group read different bank
 * slots at every diagonal where the relation allows (a fixed order: the row sums change only
 * by rounding, deterministically). */
int dg_staged_block(const int32_t* lrowptr, const int32_t* lcol, const float* lval, int32_t n_lanes,
                    const int32_t* rlw, int32_t n_cols, int32_t* pairs);

/* --------------------------------------------------------------------------------------
 * GCN epilogue (T4 tail + T5 + T6):  for one node type i with groups g = (i, j_1..j_m),
 *
 *     s_g[r]   = sum_{c < n_chunks_g} partial_g[c][r][:]              (chunk order)
 *     y_g[r]   = s_g[r] * rsqrt(max(sum(s_g[r]^2), 1e-12))            if DG_EPI_L2NORM
 *     out[r]   = act( sum_g y_g[r] )                                  (group order)
 *
 * act = relu if DG_EPI_RELU.  With DG_EPI_CHUNK_RELU each chunk partial is passed through
 * relu before the chunk sum (a layer built with act=relu and chunk = 1 applies the
 * activation per relation before add_n, layers.py:91).  With one group and no flags this is
 * the plain chunk reduce used before the cross-GPU all-reduce.
 * Replaces: tf.nn.l2_normalize(outputs, dim=1)   layers.py:93, :117
 *           tf.nn.relu(tf.add_n(hid1))           model.py:75
 *           tf.add_n(embeds)                     model.py:88
 * -------------------------------------------------------------------------------------- */
#define DG_EPI_L2NORM 1
#define DG_EPI_RELU 2
#define DG_EPI_CHUNK_RELU 4

typedef struct dg_epi_group {
    const float* partial;       /* device, [n_chunks][n_rows][d] */
    float* sum_out;             /* device, [n_rows][d]: the group's pre-normalisation sum
                                   S_ij (what the backward of l2_normalize needs), or NULL */
    int32_t n_chunks;
    int32_t group_flags;        /* 0, or DG_EPI_PUSH (dg_gcn_epilogue_peer_f32 only): sum_out also
                                 * stored into every peer's copy — the rank's slot of the peer
                                 * all-reduce of the sums (ABI 34) */
} dg_epi_group;

int dg_gcn_epilogue_f32(const dg_epi_group* groups /* HOST array */, int32_t n_groups,
                        float* out, int32_t n_rows, int32_t d, int32_t flags, void* stream);

/* Several node types' epilogues in one launch (every target's rows finish side by side; the
 * groups of all targets together at most DG_MAX_GROUPS).  Same flags for all targets. */
#define DG_EPI_MAX_TARGETS 8
typedef struct dg_epi_target {
    const dg_epi_group* groups; /* HOST array of n_groups                                   */
    int32_t n_groups;
    int32_t reserved0;
    float* out;                 /* device, [n_rows][d], 16-byte aligned                     */
    int32_t n_rows;
    int32_t target_flags;       /* 0, or DG_EPI_PUSH (dg_gcn_epilogue_peer_f32 only)        */
    int32_t reserved[2];
} dg_epi_target;

int dg_gcn_epilogue_multi_f32(const dg_epi_target* targets /* HOST array */, int32_t n_targets,
                              int32_t d, int32_t flags, void* stream);

/* The row-table form (round 5): the same rows, sums and order — bitwise the multi form's rows —
 * from a host-built descriptor per output row (decagon_amd/kernels.py: PreparedEpilogueTab), so
 * a wave issues every group's partial loads at once.  Row i of the table: rows[i].out + off is
 * the output row (its target's output base in .out); group g < (info & 7) <= 4 has
 * (n_chunks >> 8g) & 0xff chunk partials at part[g] + c * plane; info bit 8: with xchg, the row
 * also goes to every peer's copy of .out (bytes = the target's output size).  No group sums
 * (dg_epi_group.sum_out).  d = 32 or 64; rows 64-byte aligned; xchg as dg_gcn_epilogue_peer_f32
 * (the launch then ends with the exchange), or NULL. */
typedef struct dg_epi_row_desc {
    float* out;
    const float* part[4];
    int32_t off;
    int32_t plane;
    uint32_t n_chunks;
    uint32_t info;
    int32_t bytes;
    int32_t pad;
} dg_epi_row_desc;        /* 64 bytes */

struct dg_peer_xchg;
int dg_gcn_epilogue_tab_f32(const dg_epi_row_desc* rows, int32_t n_rows, int32_t d, int32_t flags,
                            const struct dg_peer_xchg* xchg /* HOST, or NULL */, void* stream);

/* --------------------------------------------------------------------------------------
 * Peer-store exchange over xGMI: the all-gather of the row-split blocks of the sharded
 * forward (decagon_amd/sharding.py; one per layer, made necessary by the normalisation of
 * the full per-(i,j) sum, layers.py:92-93), without RCCL.
 *
 * Every rank holds the row-split outputs of a layer in ONE exchange region of the same layout
 * on every rank (its own rows block `rank`); each rank maps every peer's region (IPC) and
 * stores its finished rows straight into them, write-through at system scope.  The launch's
 * last workgroup then stores the slot's epoch into word [slot][rank] of every peer's flag
 * block (uncached memory) and waits — bounded by timeout_ticks of the 100 MHz s_memrealtime
 * clock — until every rank's epoch for the slot has arrived in its own block; the kernels
 * that read the gathered rows start after that launch ends.  A wait that times out sets the
 * error word state[DG_PEER_ERROR_WORD] (0x10000 | slot << 8 | source rank) and returns; once
 * it is set, every later wait returns at once (the host checks the word and raises).
 * state: this rank's device words (DG_PEER_STATE_WORDS), zeroed once: per slot {arrivals, epoch},
 * then the error word; from DG_PEER_SUB_BASE, 8 arrival sub-counters per slot, DG_PEER_SUB_STRIDE
 * words apart (launches of >= 128 workgroups count their arrivals in two levels).
 * A slot's launches must all use the same grid (the arrival count), and every rank must run
 * the same sequence of exchanges per slot.
 * Replaces: the RCCL/NCCL all-gather of the sharded step (the reference has no parallelism).
 * -------------------------------------------------------------------------------------- */
#define DG_PEER_MAX 8
#define DG_PEER_SLOTS 8
#define DG_PEER_SUB_BASE 64
#define DG_PEER_SUB_STRIDE 16
#define DG_PEER_STATE_WORDS (DG_PEER_SUB_BASE + DG_PEER_SLOTS * 8 * DG_PEER_SUB_STRIDE)
#define DG_PEER_ERROR_WORD (2 * DG_PEER_SLOTS)
/* Wait records (round 6), in the state words between the error word and the sub-counters.
 * The wait that times out writes, before the error word: DIAG+0 its slot, +1 the epoch it
 * expected, +2..+9 the flag word it last read from each source, +10/+11 the s_memrealtime tick
 * its wait started (low / high word), +12/+13 the tick it gave up, +14/+15 the tick this rank
 * raised its own flags.  Every wait that completes after more than DG_PEER_SLOW_TICKS adds 1 to
 * +16 and max-updates +17 with its ticks (a completed wait costs one compare otherwise).  A
 * host that finds the error word reads these and, with dg_peer_read, the flag words as they
 * stand now: a late source's flag that has since reached the expected epoch was late (a host or
 * scheduling skew longer than the bound); one still short of it was never raised. */
#define DG_PEER_DIAG_BASE 24
#define DG_PEER_DIAG_WORDS 18
#define DG_PEER_SLOW_TICKS 10000 /* 100 µs */
#define DG_IPC_HANDLE_BYTES 64
#define DG_EPI_PUSH 1           /* dg_epi_target.target_flags: push this target's rows          */

typedef struct dg_peer_xchg {
    int64_t delta[DG_PEER_MAX];   /* bytes from this rank's exchange region to rank p's region as
                                     mapped in this process (delta[rank] = 0; 16-byte multiples) */
    uint32_t* flags[DG_PEER_MAX]; /* rank p's flag block [DG_PEER_SLOTS][DG_PEER_MAX], mapped here */
    uint32_t* state;              /* device, DG_PEER_STATE_WORDS words of THIS rank, zeroed once  */
    int64_t timeout_ticks;        /* > 0: s_memrealtime ticks (100 MHz) a wait may spin           */
    int32_t rank, world;          /* 1 <= world <= DG_PEER_MAX                                    */
    int32_t slot;                 /* < DG_PEER_SLOTS                                              */
    int32_t loopback;             /* 1: one-GPU rehearsal — every "peer" region is local scratch, */
                                  /* flags[p] all this rank's block, and the last workgroup raises */
                                  /* word [slot][p] for every p itself                             */
} dg_peer_xchg;

/* Device memory for the exchange: kind 0 = hipMalloc-like (coarse-grained), 1 = fine-grained,
 * 2 = uncached (the flag blocks).  Zero-filled.  These two are the library's only allocating
 * entry points; the memory is the caller's to free with dg_peer_free. */
int dg_peer_alloc(int64_t bytes, int32_t kind, void** ptr /* HOST out */);
int dg_peer_free(void* ptr);
/* IPC: the handle (DG_IPC_HANDLE_BYTES, host) of the allocation holding ptr and ptr's byte
 * offset in it; open / close a peer process's handle in this process. */
int dg_ipc_get_handle(void* ptr, void* handle /* HOST out */, int64_t* offset /* HOST out */);
int dg_ipc_open(const void* handle /* HOST */, void** ptr /* HOST out */);
int dg_ipc_close(void* ptr);
/* Synchronous copy of `bytes` of device memory (a flag block) to the host: the timeout record's
 * "flag words now" read (decagon_amd/peer.py PeerExchange.diagnostics). */
int dg_peer_read(const void* device, void* host /* HOST out */, int64_t bytes);

/* Stand-alone exchange: push bytes [offsets[s], offsets[s] + sizes[s]) of this rank's region
 * (its blocks) into every peer's region at the same offsets, then raise / wait as above. */
int dg_peer_allgather(const dg_peer_xchg* xchg /* HOST */, const void* region, const int64_t* offsets /* HOST */,
                      const int64_t* sizes /* HOST */, int32_t n_seg, void* stream);

/* dg_gcn_epilogue_multi_f32 that also pushes the rows of every target with DG_EPI_PUSH (its
 * `out` inside the exchange region) to every peer and ends with the exchange: the finishing
 * launch of a row-split layer and its all-gather in one kernel. */
int dg_gcn_epilogue_peer_f32(const dg_epi_target* targets /* HOST array */, int32_t n_targets, int32_t d,
                             int32_t flags, const dg_peer_xchg* xchg /* HOST */, void* stream);

/* dg_gcn_fused_seg_f32 whose every target's `out` lies in the exchange region: the rows are
 * also pushed to every peer and the launch ends with the exchange (config S at N = 2: a
 * layer and its all-gather in one kernel). */
int dg_gcn_fused_seg_peer_f32(const dg_seg_group* groups /* HOST */, int32_t n_groups,
                              const dg_fused_target* targets /* HOST */, int32_t n_targets, int32_t d_in,
                              int32_t d_out, const dg_peer_xchg* xchg /* HOST */, void* stream);

/* --------------------------------------------------------------------------------------
 * Batched strided fp32 GEMM on the f32-input MFMA (v_mfma_f32_32x32x2_f32, exact fp32):
 *
 *   C_b[m][n] = sc[n] * sum_k (sa[k] * A_b[m][k]) * B_b[k][n]        b < batch
 *
 * Element (m,k) of A_b is A[b*a_bs + m*a_sm + k*a_sk]; likewise B (k,n) and C (m,n).
 * sa / sc are optional (NULL = ones).  If b_map is non-NULL, batch b reads B at
 * b + b_map[b]*b_bs and writes C at c + b_map[b]*c_bs (a rank's relation shard of a
 * relation-indexed stack).  No alignment requirement.
 * Replaces: tf.matmul(x, weights_k)                          layers.py:113 (batched over k)
 *           tf.matmul chain row·L·G·L·colᵀ (predict)         optimizer.py:87-106
 * -------------------------------------------------------------------------------------- */
typedef struct dg_gemm_desc {
    const float* a;
    const float* b;
    float* c;
    const float* sa;            /* [K] or NULL */
    const float* sc;            /* [N] or NULL */
    const int32_t* b_map;       /* [batch] or NULL */
    int64_t a_bs, a_sm, a_sk;
    int64_t b_bs, b_sk, b_sn;
    int64_t c_bs, c_sm, c_sn;
    int32_t m, n, k, batch;
    int32_t reduce;             /* 0, or R > 0: batch-reduce mode (below; b_map maps B and the mask) */
    uint32_t drop_tag;          /* batch-reduce with dropout: mask stream tag */
    const uint64_t* drop_state; /* NULL, or the device dropout state {seed, step} (below) */
    float drop_keep;            /* keep probability when drop_state != NULL */
    int32_t reserved;
} dg_gemm_desc;

int dg_gemm_f32(const dg_gemm_desc* descs /* HOST array */, int32_t n_desc, void* stream);
/* n_desc <= DG_MAX_GROUPS independent GEMMs in one launch (e.g. every (i,j) group's
 * layer-2 projection).
 * Batch-reduce mode (reduce = R > 0): the batches are summed in runs of R consecutive
 * batches (in batch order) and run q's sum is written at c + q*c_bs, q < ceil(batch / R):
 *     C_q = Σ_{b in [qR, min(qR+R, batch))} A_b·B_b
 * — the backward's Σ_k dP_k·W_kᵀ (gradient of the per-relation projections, layers.py:113)
 * as partial sums that dg_gcn_epilogue_f32 (no flags) adds up.  With drop_state != NULL each
 * batch product is first multiplied element-wise by its dropout mask (mask element
 * (b·m + row)·n + col of stream drop_tag, scaled by 1/keep, as dg_dropout_elems_f32 draws it):
 *     C_q = Σ_b M_b∘(A_b·B_b)   — the gradient through tf.nn.dropout (layers.py:112).
 * With b_map in batch-reduce mode, batch b reads B at b_map[b] and takes the mask of batch
 * b_map[b] (a rank's relation shard: local batch b is global relation b_map[b]); A and the run
 * index are not mapped. */

/* Batched Aᵀ·B over a long reduction (the weight gradient H_jᵀ·dP_k, backward of
 * layers.py:113):  C_b[m][n] = Σ_{r < rows} A[b*a_bs + r*lda + m] · B[b*b_bs + r*ldb + n],  C
 * contiguous [batch][M][N].  M, N multiples of 32 with (M/32)(N/32) <= 4.  With n_split > 1
 * the rows are cut into n_split ranges whose partials ([n_split][batch][M][N], caller's
 * 16-byte aligned `partial`) are then summed in range order. */
int dg_gemm_tn_f32(const float* a, int64_t lda, int64_t a_bs, const float* b, int64_t ldb, int64_t b_bs,
                   float* c, int32_t rows, int32_t M, int32_t N, int32_t batch, int32_t n_split,
                   float* partial, void* stream);

/* --------------------------------------------------------------------------------------
 * Edge decoder scores (T8 + T9):  for pair p,
 *     u = row_table[row_idx[p]],  v = col_table[col_idx[p]]       (rows of length d)
 *     out[p] = sum_j ( sum_k u[k] l[k] G[k][j] ) l[j] v[j]         (= uᵀ·L·G·L·v)
 * G is dense d×d row-major; l is the diagonal of L (NULL = identity).  This is the diagonal
 * of the reference's B×B product, computed without forming it.
 * Replaces: batch_predict + tf.diag_part   optimizer.py:51-57, :63-85
 * Requirements: d % 32 == 0, d <= 256.
 * -------------------------------------------------------------------------------------- */
int dg_decoder_score_f32(const float* row_table, int64_t ld_row, const float* col_table,
                         int64_t ld_col, const int32_t* row_idx, const int32_t* col_idx,
                         int32_t n_pairs, const float* G, const float* l, int32_t d,
                         float* out, void* stream);

/* bf16 DEDICOM scores (BASELINE config 5): for pair p of relation k = rel_idx[p] (rel_idx
 * NULL: k = 0), u = row_table[row_idx[p]], v = col_table[col_idx[p]] (bf16 rows),
 *     out[p] = sum_n ( sum_i bf16(u_i * l_k[i]) * G[i][n] ) * l_k[n] * v_n     (fp32 accumulation)
 * G: bf16 d×d row-major (DEDICOM's global R); l_table: bf16 [n_rel][d] diagonals D_k (NULL =
 * identity).  Pairs may mix relations.  d ∈ {64, 128, 256}; tables 16-byte aligned rows.
 * Replaces batch_predict (optimizer.py:63-85) for DEDICOM relations (model.py:130-134). */
int dg_decoder_score_bf16(const uint16_t* row_table, int64_t ld_row, const uint16_t* col_table,
                          int64_t ld_col, const int32_t* row_idx, const int32_t* col_idx,
                          const int32_t* rel_idx, int32_t n_pairs, const uint16_t* G,
                          const uint16_t* l_table, int32_t d, float* out, void* stream);

/* The same scores for config 5's layout: pairs p < n_half and p + n_half (a positive and its
 * negative, optimizer.py:37-57 — the negative replaces the row) share the column and the
 * relation, so col_idx / rel_idx are read for the first half only (row_idx, out hold 2*n_half
 * entries).  The shared side is contracted once: T = G·bf16(l_k ∘ v) on the bf16 MFMA (fp32
 * accumulation), then out[p] = sum_i u_p[i] l_k[i] T[i] and out[p + n_half] = sum_i u_n[i] l_k[i] T[i]
 * in fp32 — half the MFMA work of scoring the two pairs apart.  The bf16 operand rounding sits
 * on l_k∘v instead of u∘l_k, so the scores agree with dg_decoder_score_bf16 to bf16 operand
 * rounding.  G must be 16-byte aligned.  n_row_table / n_col_table: the tables' row counts
 * (every index must be below them); tables whose byte offsets exceed 31 bits take the 64-bit
 * addressed kernel (ABI 34). */
int dg_decoder_score_bf16_paired(const uint16_t* row_table, int64_t ld_row, int64_t n_row_table,
                                 const uint16_t* col_table, int64_t ld_col, int64_t n_col_table,
                                 const int32_t* row_idx, const int32_t* col_idx,
                                 const int32_t* rel_idx, int32_t n_half, const uint16_t* G,
                                 const uint16_t* l_table, int32_t d, float* out, void* stream);

/* Config 5's whole step in one launch: every relation slot's positive batch, its sampled
 * negatives and the hinge loss.  For local slot s < n_slots (relation slot0 + s) and i < batch,
 * p = s*batch + i:
 *     neg_rows[p]            = draw slot0*batch + p of slot (slot0+s)'s alias table
 *                              (alias_table + (slot0+s)*alias_stride entries; stride 0: one
 *                              shared table) — exactly dg_unigram_sample_slots' draws;
 *     out[p]                 = score(pos_rows[p], pos_cols[p]),
 *     out[n_slots*batch + p] = score(neg_rows[p], pos_cols[p])     (dg_decoder_score_bf16_paired,
 *                              D_k = l_table[slot0 + s]);
 *     loss[0]                = sum_p relu(out[nh + p] - (out[p] - margin))   (per-workgroup sums
 *                              in a fixed order, added in block order: deterministic).
 * workspace: DG_HINGE_WS_BYTES bytes, 16-byte aligned, first word zero before the first call
 * (left zero).  d == 256; G, tables and l_table 16-byte aligned.  Replaces optimizer.py:38-47
 * (fixed_unigram_candidate_sampler over the relation's degrees), :51-57 / :63-85 (batch_predict,
 * G = R, L = D_k: model.py:130-134) and :116-120 (_hinge_loss).  n_row_table / n_col_table:
 * the tables' row counts (range <= n_row_table), as for dg_decoder_score_bf16_paired. */
int dg_slot_score_hinge_bf16(const uint16_t* row_table, int64_t ld_row, int64_t n_row_table,
                             const uint16_t* col_table, int64_t ld_col, int64_t n_col_table,
                             const int32_t* pos_rows, const int32_t* pos_cols,
                             const uint32_t* alias_table, int32_t range, int64_t alias_stride,
                             int32_t slot0, int32_t n_slots, int32_t batch, uint64_t seed,
                             const uint16_t* G, const uint16_t* l_table, int32_t d, float margin,
                             float* out, int32_t* neg_rows, float* loss, void* workspace, void* stream);

/* Fused decoder step (T8 + T9 + T11 + T12 in one launch):
 *   neg_row[b] = neg_rows[b] if neg_rows != NULL, else draw (offset + b) of the alias
 *                sampler — the same draws as dg_unigram_sample — written to neg_rows_out[b]
 *                if non-NULL;
 *   pos[b] = score(rows[b], cols[b]);  neg[b] = score(neg_row[b], cols[b])   (as above)
 *   loss[0] = sum_b relu(neg[b] - (pos[b] - margin))   (fixed block order)
 * workspace: device, 16-byte aligned, 16 + 4*ceil(n/32) bytes, all zero before the first
 * call (the kernel leaves it so).  n >= 1.  The partial sums of the 32-pair blocks meet in one
 * returning 64-bit integer atomic per block (fixed point, each partial rounded to the nearest
 * 2^-32: the loss is within 255·2^-33 ≈ 3e-8 absolute of the sum of the fp32 partials; integer
 * adds are order-free, so bitwise reproducible) when there are at most 255 blocks, else
 * through a ticket and block-order reads (the fp32 partials in block order).
 * Replaces optimizer.py:37-57 (sampler, gathers, pos/neg scores) + :116-120 (hinge). */
int dg_decoder_hinge_f32(const float* row_table, int64_t ld_row, const float* col_table,
                         int64_t ld_col, const int32_t* rows, const int32_t* cols,
                         const int32_t* neg_rows, const uint32_t* alias_table, int32_t range,
                         uint64_t seed, uint64_t offset, int32_t n, const float* G,
                         const float* l, int32_t d, float margin, float* pos, float* neg,
                         int32_t* neg_rows_out, float* loss, void* workspace, void* stream);

/* Hinge loss (T12):  loss[0] = sum_p relu(neg[p] - pos[p] + margin).
 * Replaces DecagonOptimizer._hinge_loss  optimizer.py:116-120.  Single workgroup,
 * fixed summation order. */
int dg_hinge_loss_f32(const float* pos, const float* neg, int32_t n, float margin,
                      float* loss, void* stream);

/* The same hinge sum over many pairs (config 5: every slot's batch, 10^6 pairs) on up to
 * DG_HINGE_WS_BLOCKS workgroups, partials added in block order (deterministic for a given n).
 * workspace: device, 16-byte aligned, DG_HINGE_WS_BYTES bytes, its first word zero before the
 * first call (the kernel leaves it zero again).  optimizer.py:116-120. */
#define DG_HINGE_WS_BLOCKS 256
#define DG_HINGE_WS_BYTES (16 + 4 * DG_HINGE_WS_BLOCKS)
int dg_hinge_loss_ws_f32(const float* pos, const float* neg, int32_t n, float margin, float* loss,
                         void* workspace, void* stream);

/* Cross-entropy loss:  loss[0] = sum_p softplus(-pos[p]) + w * sum_p softplus(neg[p])
 * (sigmoid_cross_entropy_with_logits with labels 1 / 0).  optimizer.py:122-127. */
int dg_xent_loss_f32(const float* pos, const float* neg, int32_t n, float neg_weight,
                     float* loss, void* stream);

/* --------------------------------------------------------------------------------------
 * Training step (backward of the hinge cost + TF Adam), optimizer.py:108-114.
 * -------------------------------------------------------------------------------------- */
/* Decoder gradient for the n positive pairs (rows[p], cols[p]) and negatives (neg_rows[p],
 * cols[p]) whose scores pos / neg the forward produced (dg_decoder_hinge_f32): with
 * a_p = [neg[p] - (pos[p] - margin) > 0] and M = L·G·L (L = diag(l), NULL = I),
 *     grad_rows[p] = -a_p·M·v_p,  grad_rows[n + p] = a_p·M·v_p,  grad_cols[p] = a_p·Mᵀ·(un_p - u_p)
 *     dM = Σ_p a_p·(un_p - u_p)·v_pᵀ;   dG = L·dM·L   (if dG != NULL)
 *     dl[a] = Σ_b dM[a][b]G[a][b]l[b] + Σ_c dM[c][a]G[c][a]l[c]   (if dl != NULL; needs l)
 *     dG_diag[a] = dG[a][a]                                      (if dG_diag != NULL)
 * grad_rows is [2n][d], grad_cols [n][d] (dense rows; dg_scatter_rows_f32 adds them into the
 * embedding gradients).  workspace: 16-byte aligned, dg_decoder_grad_workspace(n, d) bytes.
 * d % 32 == 0, d <= 256.  Replaces the gradient of optimizer.py:51-57, :63-85, :116-120. */
int64_t dg_decoder_grad_workspace(int32_t n, int32_t d);
int dg_decoder_grad_f32(const float* row_table, int64_t ld_row, const float* col_table,
                        int64_t ld_col, const int32_t* rows, const int32_t* cols,
                        const int32_t* neg_rows, int32_t n, const float* pos, const float* neg,
                        const float* G, const float* l, int32_t d, float margin,
                        float* grad_rows, float* grad_cols, float* dG, float* dl, float* dG_diag,
                        void* workspace, int64_t workspace_bytes, void* stream);

/* out[idx[q]][:] += Σ_{q' : idx[q'] = idx[q]} src[q'][:]  (occurrences summed in q' order,
 * each distinct row written once).  The gradient of tf.gather (optimizer.py:66-76).
 * d <= 256; indices outside [0, n_out_rows) update nothing (device-side guard: the
 * indices may be sampled on the device, where the host cannot check them). */
int dg_scatter_rows_f32(const int32_t* idx, int32_t n, const float* src, int32_t d, float* out,
                        int64_t ld_out, int32_t n_out_rows, void* stream);

/* Backward of y_g = l2_normalize(s_g) for every group g of one node type (layers.py:93,
 * :117; model.py:75): dy' = dy ∘ [mask > 0] (mask = the relu output, or NULL), then
 *     ds_g = dy'·inv − s_g·inv³·(s_g·dy')·[Σs_g² >= 1e-12],   inv = rsqrt(max(Σs_g², 1e-12))
 * (tf.maximum passes its gradient to Σs² where Σs² >= ε).  All rows [n_rows][d], 16-byte
 * aligned; d % 4 == 0, d <= 256. */
typedef struct dg_l2g_group {
    const float* s;             /* [n_rows][d] the pre-normalisation sum (forward) */
    float* ds;                  /* [n_rows][d] its gradient (output) */
} dg_l2g_group;

int dg_l2norm_grad_f32(const dg_l2g_group* groups /* HOST array */, int32_t n_groups,
                       const float* dy, const float* mask, int32_t n_rows, int32_t d,
                       void* stream);

/* TF 1.8 ApplyAdam (use_nesterov = false) on up to DG_MAX_ADAM_SEGS segments in one launch:
 *     m += (g − m)(1 − β1);  v += (g² − v)(1 − β2);  param −= alpha·m / (sqrt(v) + ε)
 * alpha = lr·sqrt(1 − β2^t)/(1 − β1^t): read from state[2] when `state` (device, float[3] =
 * {β1^t, β2^t, alpha}) is non-NULL — graph-capturable, advanced on the device by
 * dg_adam_advance after the update, as TF's _finish advances its beta-power variables —
 * else the `alpha` argument.  grad NULL = a zero gradient (TF updates every variable each
 * step).  16-byte aligned.  Initial state: {β1, β2, lr·sqrt(1 − β2)/(1 − β1)}. */
#define DG_MAX_ADAM_SEGS 32

typedef struct dg_adam_seg {
    float* param;
    const float* grad;          /* or NULL */
    float* m;
    float* v;
    int64_t n;
} dg_adam_seg;

int dg_adam_f32(const dg_adam_seg* segs /* HOST array */, int32_t n_segs, float alpha, float beta1,
                float beta2, float eps, const float* state, void* stream);
int dg_adam_advance(float* state, float lr, float beta1, float beta2, void* stream);

/* --------------------------------------------------------------------------------------
 * Dropout (training path): dropout_sparse (layers.py:23-31, :88) and tf.nn.dropout (:112).
 * state: device uint64 {seed, step}.  Element idx of stream `tag` is kept iff
 *   lowbias32(key ^ idx) >> 8 < (uint32)(keep·2^24),
 *   key = lowbias32(lowbias32(seed_lo ^ tag·0x9E3779B9) ^ (seed_hi + step·0x85EBCA6B)),
 *   lowbias32(x): x ^= x>>16; x *= 0x7feb352d; x ^= x>>15; x *= 0x846ca68b; x ^= x>>16,
 * and a kept element is scaled by 1/keep (TF's distribution; its RNG stream is not
 * reproducible).  dg_dropout_advance increments step (a new draw per training step, on the
 * device: graph-capturable).
 * -------------------------------------------------------------------------------------- */
/* out[r][:] = in[r][:] · s(r)  (row masks: identity features' dropout_sparse, one relation's
 * rows at a time in the relation-stacked W1; in place allowed).  n_rows·d < 2^32. */
int dg_dropout_rows_f32(const float* in, float* out, int64_t n_rows, int32_t d, const uint64_t* state,
                        uint32_t tag, float keep, void* stream);
/* out[k][r][f] = src[r][f] · s(k·n_rows·d + r·d + f)  for k < K: tf.nn.dropout of H_j drawn
 * independently for each of the K relations.  K·n_rows·d < 2^32. */
int dg_dropout_elems_f32(const float* src, float* out, int32_t K, int32_t n_rows, int32_t d,
                         const uint64_t* state, uint32_t tag, float keep, void* stream);
/* Relation-mapped forms for a rank's relation shard (sharding.py): local slab b is global
 * relation rel_map[b] and draws THAT relation's mask bits (the bits the unmapped forms draw
 * for it).  Rows: slab b is rows_per_slab rows; flags bit 1 / bit 2 address `in` / `out` at
 * slab rel_map[b] (else b).  Elems: out[b] = src ∘ M_{rel_map[b]} (out local, contiguous). */
int dg_dropout_rows_map_f32(const float* in, float* out, const int32_t* rel_map, int32_t n_map,
                            int64_t rows_per_slab, int32_t d, int32_t flags, const uint64_t* state,
                            uint32_t tag, float keep, void* stream);
int dg_dropout_elems_map_f32(const float* src, float* out, const int32_t* rel_map, int32_t K,
                             int32_t n_rows, int32_t d, const uint64_t* state, uint32_t tag, float keep,
                             void* stream);
int dg_dropout_advance(uint64_t* state, void* stream);

/* --------------------------------------------------------------------------------------
 * Evaluation: AUROC, AUPRC and AP@k of n_pos positive vs n_neg negative edge
 * scores, exactly as roc_auc_score (ties count ½), average_precision_score and
 * rank_metrics.apk(actual = positives, predicted = all sorted by score, stable, descending)
 * compute them in get_accuracy_scores (main.py:38-80): out[0..2] = {auroc, auprc, apk}
 * (double).  Integer pair counts per positive, no sort; workspace 16-byte aligned,
 * dg_rank_metrics_workspace(n_pos) bytes.
 * -------------------------------------------------------------------------------------- */
int64_t dg_rank_metrics_workspace(int32_t n_pos);
int dg_rank_metrics_f32(const float* pos, int32_t n_pos, const float* neg, int32_t n_neg, int32_t k,
                        double* out, void* workspace, int64_t workspace_bytes, void* stream);

/* The same metrics of the scores the reference actually ranks: mode DG_RANK_SIGMOID64 =
 * main.py:51-52,60,70,81 under numpy 1.14 (requirements.txt:14) — float32 exp of TF's float32
 * logit (correctly rounded, as glibc expf), float64 `1. / (1 + e)`, np.nan_to_num — so logits
 * above ≈36.7 / below ≈-88.7 tie at 1.0 / 0.0; DG_RANK_SIGMOID32 = MathUtils.sigmoid on the
 * float32 decoder output (DecagonAccuracyEvaluator.py:123, all float32); DG_RANK_LOGIT = the
 * logits (as dg_rank_metrics_f32).  pos / neg are the LOGITS.  Workspace 16-byte aligned,
 * dg_rank_metrics_ex_workspace(n_pos, n_neg) bytes. */
#define DG_RANK_LOGIT 0
#define DG_RANK_SIGMOID64 1
#define DG_RANK_SIGMOID32 2
int64_t dg_rank_metrics_ex_workspace(int32_t n_pos, int32_t n_neg);
int dg_rank_metrics_ex_f32(const float* pos, int32_t n_pos, const float* neg, int32_t n_neg, int32_t k,
                           int32_t mode, double* out, void* workspace, int64_t workspace_bytes, void* stream);

/* --------------------------------------------------------------------------------------
 * Unigram negative sampler (T11):  out[i] ~ Categorical(p), p_c ∝ degree_c^0.75, draw
 * (offset + i) of a counter-based hash stream, through a Walker alias table of `range`
 * entries {acceptance probability as float bits, alias index} (uint32 pairs, built once on
 * the host: decagon_amd/sampling.py).
 * Replaces tf.nn.fixed_unigram_candidate_sampler(distortion=0.75, unique=False)
 * optimizer.py:40-47 (distribution only — TF's RNG stream is not reproducible).
 * -------------------------------------------------------------------------------------- */
int dg_unigram_sample(const uint32_t* alias_table, int32_t range, int32_t n, uint64_t seed,
                      uint64_t offset, int32_t* out, void* stream);

/* The same draws with one table per relation slot (optimizer.py:38-47 samples relation k's
 * negatives from ITS degrees, degrees[i][k]): draw i < n is draw slot0*batch + i of the table
 * of slot slot0 + i / batch, at alias_table + (slot0 + i / batch) * alias_stride entries
 * (alias_stride 0: one shared table, = dg_unigram_sample with offset slot0*batch). */
int dg_unigram_sample_slots(const uint32_t* alias_table, int32_t range, int64_t alias_stride,
                            int32_t slot0, int32_t batch, int32_t n, uint64_t seed, int32_t* out,
                            void* stream);

#ifdef __cplusplus
}
#endif

#endif /* DECAGON_HIP_H */
