"""Config 5 (BASELINE configs[4]): bf16 DEDICOM scoring of every drug-drug relation slot's
negative-sampled batch, in one launch, sharded by slot across GPUs.

The reference scores one relation's minibatch per training step: the negatives come from
`fixed_unigram_candidate_sampler` over THAT relation's degrees (degree^0.75,
optimizer.py:38-47), the positive and negative scores from `batch_predict` with G = R (global
interaction) and L = D_k (the relation's local variation, model.py:130-134, optimizer.py:51-57),
and the cost from `_hinge_loss` (optimizer.py:116-120).  Config 5 runs that for all slots at
once with d = 256 bf16 embeddings and parameters (fp32 accumulation), in two launches:

  1. dg_slot_scores_bf16: each slot's B negatives drawn from the slot's own alias table (draw
     i of slot s is counter s·B + i, so the draws do not depend on how the slots are sharded),
     then per slot T_k = E·(D_k∘R) for every drug (32-row tiles on the bf16 MFMA) and each of
     the slot's 2B pairs scored as T_k[u]·(D_k∘v);
  2. dg_hinge_loss_ws_f32 sums relu(neg − pos + margin) over the rank's pairs, and
  3. with N ranks, one all-reduce of that scalar — the only collective.

Slots are dealt in contiguous blocks (sharding.slot_range); embeddings and parameters are
replicated (645 × 256 bf16 = 330 KB; the slots' alias tables 1,928 × 645 × 8 B = 10 MB).
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import torch

from . import kernels


class SlotScorer:
    def __init__(self, E_row: torch.Tensor, E_col: torch.Tensor, R: torch.Tensor, D: torch.Tensor,
                 pos_rows: torch.Tensor, pos_cols: torch.Tensor, alias: torch.Tensor, batch: int,
                 margin: float = 0.1, seed: int = 11, slots: Optional[Tuple[int, int]] = None,
                 allreduce: Optional[Callable[[torch.Tensor], None]] = None):
        """E_row / E_col: bf16 [n, d] embeddings; R: bf16 [d, d]; D: bf16 [n_slots, d]
        diagonals; pos_rows / pos_cols: int32 [n_slots·batch] positive pairs of every slot
        (slot-major); alias: the slots' degree^0.75 alias tables (kernels.upload_alias of a
        list of degree vectors: [n_slots, range, 2]; a single [range, 2] table is shared by
        every slot); slots: this rank's [s0, s1) (default: all).  R is read through its
        transpose, made here: call refresh() after changing R in place."""
        n_slots = D.shape[0]
        if pos_rows.numel() != n_slots * batch or pos_cols.numel() != n_slots * batch:
            raise ValueError("pos_rows / pos_cols must hold n_slots * batch pairs")
        s0, s1 = (0, n_slots) if slots is None else slots
        if not 0 <= s0 <= s1 <= n_slots:
            raise ValueError("slot range outside [0, n_slots]")
        rng = alias.shape[-2]
        if rng > E_row.shape[0]:
            raise ValueError("sampler range exceeds the row table")
        if alias.dim() == 3 and alias.shape[0] != n_slots:
            raise ValueError("one alias table per slot expected")
        dev = E_row.device
        self.s0, self.s1, self.batch, self.seed, self.margin = s0, s1, batch, seed, float(margin)
        n = (s1 - s0) * batch
        self.n = n
        self.pos_rows = pos_rows[s0 * batch:s1 * batch].to(torch.int32).contiguous()
        self.pos_cols = pos_cols[s0 * batch:s1 * batch].to(torch.int32).contiguous()
        self.neg_rows = torch.empty(n, dtype=torch.int32, device=dev)
        self.out = torch.empty(2 * n, dtype=torch.float32, device=dev)   # pos scores, then neg
        self.loss = torch.zeros(1, dtype=torch.float32, device=dev)
        self._ws = kernels.hinge_workspace(dev)
        self.E_row, self.E_col, self.R, self.D, self.alias = E_row, E_col, R, D, alias
        self.Rt = torch.empty_like(R)
        self.refresh()
        self.allreduce = allreduce

    def refresh(self) -> None:
        """Re-read R (its transpose is what the kernel's operands are built from)."""
        self.Rt.copy_(self.R.t())

    @property
    def pos(self) -> torch.Tensor:
        return self.out[:self.n]

    @property
    def neg(self) -> torch.Tensor:
        return self.out[self.n:]

    def score(self) -> None:
        """Sampler + scorer: one launch."""
        if self.n:
            kernels.slot_scores_bf16(self.E_row, self.E_col, self.Rt, self.D, self.pos_rows, self.pos_cols,
                                     self.batch, self.s0, self.alias, self.seed, self.neg_rows, self.out)

    def hinge(self) -> None:
        kernels.hinge_loss(self.pos, self.neg, self.margin, out=self.loss, workspace=self._ws)
        if self.allreduce is not None:
            self.allreduce(self.loss)

    def __call__(self) -> None:
        self.score()
        self.hinge()
