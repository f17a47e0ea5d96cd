"""Tower placement: the reference TF variant's MPMD split, on RCCL ranks.

The reference places the positive doc tower on /gpu:0, negative k on /gpu:k and the
query tower + cosine/softmax head on /cpu:0, with TF moving vectors and gradients
between devices implicitly (dssm_cnn_v2/cnn_dssm_tf.py:139-176).  Here the S = 1+J
document *slots* are distributed over the ranks instead (rank r encodes slots r, r+W,
...; S % W == 0), which is the same partition of the work with explicit collectives:

* forward: each rank runs the shared doc tower on its slots (B x S/W pages), the page
  vectors are all-gathered (RCCL over xGMI) so every rank holds all (B, S, D);
* every rank runs the (small) query tower and the explicit-negative head with the SAME
  dropout seed, so all ranks see the identical loss (metrics need no reduction);
* backward: the all-gather's reduce-scatter returns to each rank the gradient of its
  own slots; the loss is back-propagated scaled by 1/W (W identical copies of the head)
  and the flat gradient is all-reduced with SUM, which adds the per-slot doc-tower
  contributions and restores the full query-tower gradient.

DP (parallel/ddp.py) strictly dominates this mode for throughput — it exists for
parity with the reference's placement experiment and as the template for splitting a
step by tower rather than by sample.
"""
from __future__ import annotations

from typing import List, Tuple

import torch

from . import dist as pdist


def slots_for_rank(num_slots: int, world: int, rank: int) -> List[int]:
    if num_slots % world:
        raise ValueError(f"tower placement needs (1+J) % world_size == 0, got {num_slots} slots on {world} ranks")
    return list(range(rank, num_slots, world))


def placed_forward(model, q_ids: torch.Tensor, d_ids: torch.Tensor, base_seed: int
                   ) -> Tuple[torch.Tensor, torch.Tensor]:
    """Raw q (B, D) and d (B, S, D) with the doc slots computed on their owning ranks."""
    info = pdist.info()
    W, r = info.world_size, info.rank
    B, S, Ld = d_ids.shape
    mine = slots_for_rank(S, W, r)
    k = len(mine)
    training = model.training
    q = model.tower_forward("query", q_ids, training, base_seed * 2 + 1)
    ids = d_ids[:, mine].transpose(0, 1).reshape(k * B, Ld)  # slot-major
    dl = model.tower_forward("doc", ids, training, base_seed * 2 + 2 + 7919 * r)
    D = dl.shape[-1]
    g = pdist.all_gather_autograd(dl)                       # (W*k*B, D): rank w, local slot j, row b
    d = g.view(W, k, B, D).permute(2, 1, 0, 3).reshape(B, S, D)  # slot j*W + w
    return q, d


def scale_grad(x: torch.Tensor, s: float) -> torch.Tensor:
    """Value of x, gradient scaled by s."""
    return x * s + (x - x * s).detach()
