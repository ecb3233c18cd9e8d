"""Config 5 (BASELINE configs[4]): bf16 DEDICOM scoring of every drug-drug relation slot's
negative-sampled batch, in one launch, sharded by slot across GPUs.

The reference scores one relation's minibatch per training step: the negatives come from
`fixed_unigram_candidate_sampler` over THAT relation's degrees (degree^0.75,
optimizer.py:38-47), the positive and negative scores from `batch_predict` with G = R (global
interaction) and L = D_k (the relation's local variation, model.py:130-134, optimizer.py:51-57),
and the cost from `_hinge_loss` (optimizer.py:116-120).  Config 5 runs that for all slots at
once with d = 256 bf16 embeddings and parameters (fp32 accumulation):

  1. each slot's B negatives are drawn from the slot's own alias table (draw i of slot s is
     counter s·B + i, so the draws do not depend on how the slots are sharded),
  2. the n positive and n negative pairs are scored on the bf16 MFMA (a positive and its
     negative share the column and the relation: T = R·(D_k∘v) is contracted once for both),
  3. relu(neg − pos + margin) is summed over the rank's pairs — 1-3 in ONE launch,
     dg_slot_score_hinge_bf16 (fused=False: dg_unigram_sample_slots, dg_decoder_score_bf16_paired
     and dg_hinge_loss_ws_f32 as three launches, the same draws and scores), and
  4. with N ranks, one all-reduce of that scalar — the only collective.

Slots are dealt in contiguous blocks (sharding.slot_range); embeddings and parameters are
replicated (645 × 256 bf16 = 330 KB; the slots' alias tables 1,928 × 645 × 8 B = 10 MB).
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import torch

from . import kernels
from .tuning import knob


class SlotScorer:
    def __init__(self, E_row: torch.Tensor, E_col: torch.Tensor, R: torch.Tensor, D: torch.Tensor,
                 pos_rows: torch.Tensor, pos_cols: torch.Tensor, alias: torch.Tensor, batch: int,
                 margin: float = 0.1, seed: int = 11, slots: Optional[Tuple[int, int]] = None,
                 allreduce: Optional[Callable[[torch.Tensor], None]] = None, fused: Optional[bool] = None):
        """E_row / E_col: bf16 [n, d] embeddings; R: bf16 [d, d]; D: bf16 [n_slots, d]
        diagonals; pos_rows / pos_cols: int32 [n_slots·batch] positive pairs of every slot
        (slot-major); alias: the slots' degree^0.75 alias tables (kernels.upload_alias of a
        list of degree vectors: [n_slots, range, 2]; a single [range, 2] table is shared by
        every slot); slots: this rank's [s0, s1) (default: all)."""
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
        self.rows = torch.empty(2 * n, dtype=torch.int32, device=dev)   # positives, then negatives
        self.rows[:n] = pos_rows[s0 * batch:s1 * batch]
        cols = pos_cols[s0 * batch:s1 * batch].to(torch.int32)
        self.cols = torch.cat([cols, cols])                              # a negative keeps its column
        rel = torch.arange(s0, s1, dtype=torch.int32, device=dev).repeat_interleave(batch)
        self.rel = torch.cat([rel, rel])
        self.out = torch.empty(2 * n, dtype=torch.float32, device=dev)   # pos scores, then neg
        self.loss = torch.zeros(1, dtype=torch.float32, device=dev)
        self._ws = kernels.hinge_workspace(dev)
        self.E_row, self.E_col, self.R, self.D, self.alias = E_row, E_col, R, D, alias
        self.allreduce = allreduce
        # (DG_C5_FUSED=0: the three-launch form by default — A/B runs)
        self.fused = knob("DG_C5_FUSED", True) if fused is None else fused

    @property
    def neg_rows(self) -> torch.Tensor:
        return self.rows[self.n:]

    @property
    def pos(self) -> torch.Tensor:
        return self.out[:self.n]

    @property
    def neg(self) -> torch.Tensor:
        return self.out[self.n:]

    def sample(self) -> None:
        if self.n:
            kernels.unigram_sample_slots(self.alias, self.s0, self.batch, self.n, self.seed, out=self.neg_rows)

    def score(self) -> None:
        # positives then negatives, a negative keeping its positive's column and relation
        if self.n:
            kernels.decoder_score_bf16(self.E_row, self.E_col, self.rows, self.cols, self.R, self.D, self.rel,
                                       out=self.out, paired=True)

    def hinge(self) -> None:
        kernels.hinge_loss(self.pos, self.neg, self.margin, out=self.loss, workspace=self._ws)
        if self.allreduce is not None:
            self.allreduce(self.loss)

    def __call__(self) -> None:
        if not self.fused:
            self.sample()
            self.score()
            self.hinge()
            return
        if self.n:
            kernels.slot_score_hinge_bf16(self.E_row, self.E_col, self.rows[:self.n], self.cols[:self.n], self.alias,
                                          self.s0, self.s1 - self.s0, self.batch, self.seed, self.R, self.D,
                                          self.margin, self.out, self.neg_rows, self.loss, self._ws)
        else:
            self.loss.zero_()
        if self.allreduce is not None:
            self.allreduce(self.loss)
