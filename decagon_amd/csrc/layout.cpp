// Host-side layout helper for the LDS-staged SpMM (staged.hip): builds one relation's block
// of (column, value) pairs so that the 16 lanes of every ds_read_b128 lane group gather
// from 16 different bank slots at every diagonal the relation's structure allows.
//
// In the staged kernel thread i owns virtual row (lane) i of a relation and, at diagonal m,
// reads its pair's column v from the slab image, whose columns are 80 bytes apart: the
// 16-byte slot (mod the 256-byte bank row) of float4 j is (5v + j) mod 16 — a bijection of
// v & 15 ("the class of v") for every j.  A wave's ds_read_b128 is served in four
// 16-lane groups; lanes of one group reading different positions of one class serialize.
//
// Two choices are free, and both are made here, once per relation:
//  1. The diagonal of each of a lane's nonzeros (any order sums the same up to rounding): per
//     lane group, a proper edge colouring of the bipartite multigraph lanes x classes (one
//     edge per nonzero) with colours = diagonals — König: max-degree colours suffice, found
//     with alternating-path swaps.  Where a class holds more of the group's nonzeros than the
//     wave has diagonals, the surplus colours fold into diagonals where their lanes are free,
//     on the least-used class.
//  2. Which zero column a hole (a lane with no nonzero at a diagonal) reads: sixteen zero
//     columns, one per class, sit after the slab rows; all holes of a (lane group, diagonal)
//     read the one whose class no nonzero there uses (identical addresses broadcast).
// Measured on config P (simulated from the layout): gather cycles per conflict-free cycle
// 2.65 in feed order, 1.61 with round 1's per-diagonal matching, 1.50 with this colouring;
// permuting the slab rows over the classes as well (a local search) reached 1.06 but changed
// nothing measurable on the GPU (the kernel is not bound by these conflicts), so it was
// dropped.  Deterministic.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "decagon_hip.h"

namespace {

// lanes of the four ds_read_b128 groups (MI355X_MICROARCH.md §LDS)
int lane_group(int l) {
    const int h = l >> 5, q = l & 31;
    const bool g0 = q < 4 || (q >= 12 && q < 16) || (q >= 20 && q < 28);
    return 2 * h + (g0 ? 0 : 1);
}

struct Group {
    int lanes[16];       // lane indices (into the relation's lanes)
    int D = 0;           // diagonals of its wave
    int out = 0;         // its wave's pair-block offset (in pairs)
};

// One lane group's colouring: edges (member a, class k, nonzero p); returns each edge's
// diagonal in diag[].
void colour_group(int D, const std::vector<int>& ea, const std::vector<int>& ek, std::vector<int>& diag) {
    const int E = static_cast<int>(ea.size());
    int cdeg[16] = {0}, ldeg[16] = {0};
    for (int e = 0; e < E; ++e) {
        ++cdeg[ek[e]];
        ++ldeg[ea[e]];
    }
    int Dc = D;
    for (int k = 0; k < 16; ++k) Dc = std::max(Dc, cdeg[k]);
    for (int a = 0; a < 16; ++a) Dc = std::max(Dc, ldeg[a]);
    // at[v][c]: the edge of colour c at vertex v (v < 16: members, v >= 16: classes), or -1
    std::vector<int> at(32 * static_cast<size_t>(Dc), -1);
    auto A = [&](int v, int c) -> int& { return at[static_cast<size_t>(v) * Dc + c]; };
    diag.assign(E, -1);
    std::vector<int> path;
    for (int e = 0; e < E; ++e) {
        const int u = ea[e], v = 16 + ek[e];
        int fu = 0, fv = 0;
        while (A(u, fu) >= 0) ++fu;
        while (A(v, fv) >= 0) ++fv;
        int c = fu;
        if (A(v, fu) >= 0) {
            // fu is busy at v: swap colours fu <-> fv along the alternating path from v (it
            // cannot reach u in a bipartite graph), which frees fu at v
            path.clear();
            int x = v, cur = fu;
            while (A(x, cur) >= 0) {
                const int f = A(x, cur);
                path.push_back(f);
                x = (x == ea[f]) ? 16 + ek[f] : ea[f];
                cur = (cur == fu) ? fv : fu;
            }
            for (int f : path) {
                A(ea[f], diag[f]) = -1;
                A(16 + ek[f], diag[f]) = -1;
            }
            for (int f : path) {
                diag[f] = (diag[f] == fu) ? fv : fu;
                A(ea[f], diag[f]) = f;
                A(16 + ek[f], diag[f]) = f;
            }
        }
        diag[e] = c;
        A(u, c) = e;
        A(v, c) = e;
    }
    if (Dc == D) return;
    // surplus colours: each such edge moves to a diagonal < D where its lane is free (one
    // exists: the lane has at most D nonzeros and one of them sits past D), on the class used
    // least there
    std::vector<int> use(static_cast<size_t>(D) * 16, 0);
    std::vector<char> busy(static_cast<size_t>(D) * 16, 0);
    for (int e = 0; e < E; ++e)
        if (diag[e] < D) {
            ++use[static_cast<size_t>(diag[e]) * 16 + ek[e]];
            busy[static_cast<size_t>(diag[e]) * 16 + ea[e]] = 1;
        }
    for (int e = 0; e < E; ++e) {
        if (diag[e] < D) continue;
        int best = -1;
        for (int m = 0; m < D; ++m) {
            if (busy[static_cast<size_t>(m) * 16 + ea[e]]) continue;
            if (best < 0 || use[static_cast<size_t>(m) * 16 + ek[e]] < use[static_cast<size_t>(best) * 16 + ek[e]])
                best = m;
        }
        diag[e] = best;
        ++use[static_cast<size_t>(best) * 16 + ek[e]];
        busy[static_cast<size_t>(best) * 16 + ea[e]] = 1;
    }
}

}  // namespace

extern "C" int dg_staged_block(const int32_t* lrowptr, const int32_t* lcol, const float* lval, int32_t n_lanes,
                               const int32_t* rlw, int32_t n_cols, int32_t* pairs) {
    if (!lrowptr || !rlw || !pairs || n_lanes < 0 || (n_lanes & 63) || n_cols < 1 || n_cols > 1024)
        return DG_EINVAL;
    const int n_w = n_lanes / 64;
    const int nnz = lrowptr[n_lanes];
    if (nnz > 0 && (!lcol || !lval)) return DG_EINVAL;
    // groups and their pair-block offsets
    std::vector<Group> grp(static_cast<size_t>(n_w) * 4);
    int64_t off = 0;
    for (int w = 0; w < n_w; ++w) {
        int fill[4] = {0, 0, 0, 0};
        for (int l = 0; l < 64; ++l) {
            const int gi = lane_group(l);
            grp[w * 4 + gi].lanes[fill[gi]++] = 64 * w + l;
        }
        for (int gi = 0; gi < 4; ++gi) {
            grp[w * 4 + gi].D = rlw[w];
            grp[w * 4 + gi].out = static_cast<int>(off);
        }
        for (int l = 0; l < 64; ++l) {
            const int len = lrowptr[64 * w + l + 1] - lrowptr[64 * w + l];
            if (len > rlw[w]) return DG_EINVAL;
        }
        off += static_cast<int64_t>(rlw[w]) * 64;
        if (off > 0x7fffffff) return DG_EINVAL;
    }
    for (int p = 0; p < nnz; ++p)
        if (lcol[p] < 0 || lcol[p] >= n_cols) return DG_EINVAL;
    const int G = static_cast<int>(grp.size());

    // per group: colour, fold, place; holes read the zero column of a free class
    std::vector<int> ea, ek, ep, diag;
    std::vector<int> used;
    for (int g = 0; g < G; ++g) {
        const Group& gr = grp[g];
        const int D = gr.D;
        if (D == 0) continue;
        ea.clear();
        ek.clear();
        ep.clear();
        for (int a = 0; a < 16; ++a) {
            const int l = gr.lanes[a];
            for (int p = lrowptr[l]; p < lrowptr[l + 1]; ++p) {
                ea.push_back(a);
                ek.push_back(lcol[p] & 15);
                ep.push_back(p);
            }
        }
        colour_group(D, ea, ek, diag);
        used.assign(static_cast<size_t>(D), 0);  // class bit mask per diagonal
        std::vector<char> has(static_cast<size_t>(D) * 16, 0);
        for (size_t e = 0; e < ea.size(); ++e) {
            const int l = gr.lanes[ea[e]];
            const int64_t q = gr.out + static_cast<int64_t>(diag[e]) * 64 + (l & 63);
            pairs[2 * q] = lcol[ep[e]];
            memcpy(&pairs[2 * q + 1], &lval[ep[e]], 4);
            used[diag[e]] |= 1 << ek[e];
            has[static_cast<size_t>(diag[e]) * 16 + ea[e]] = 1;
        }
        for (int m = 0; m < D; ++m) {
            int z = 0;
            while (z < 15 && (used[m] >> ((n_cols + z) & 15) & 1)) ++z;
            for (int a = 0; a < 16; ++a) {
                if (has[static_cast<size_t>(m) * 16 + a]) continue;
                const int64_t q = gr.out + static_cast<int64_t>(m) * 64 + (gr.lanes[a] & 63);
                pairs[2 * q] = n_cols + z;
                pairs[2 * q + 1] = 0;
            }
        }
    }
    return DG_OK;
}
