"""Framebuffer partitioning across GPUs and the RGB8 gather.

One process per GPU (torch.distributed; backend "nccl" = RCCL over xGMI on ROCm).  Rows are
dealt in blocks of `row_block` rows round-robin over ranks (block b -> rank b % world), which
balances the load: a mesh covers only the central rows of a frame, so contiguous bands
would leave most ranks idle.  Every rank renders its rows with ceres_render_device
(ceres_tiling) into a compact local RGB8 buffer (local row k stored at position n_k - 1 - k),
and ONE collective per frame -- a gather of those buffers to rank 0 -- assembles the PPM
body there.  The scene itself is replicated (uploaded per device, outside the timed region).
The reference has no distributed code at all (render.hpp:104 is an OpenMP loop).
"""
import numpy as np


def row_map(H, row_block, world):
    """Global rows j owned by each rank, in local-row order (matches ceres_tiling)."""
    nb = (H + row_block - 1) // row_block
    out = []
    for r in range(world):
        rows = [j for b in range(r, nb, world) for j in range(b * row_block, min(H, (b + 1) * row_block))]
        out.append(np.asarray(rows, np.int64))
    return out


def ppm_row_permutation(H, row_block, world):
    """Index into the concatenation of all ranks' padded local buffers (rank-major, `maxrows`
    rows each) giving, for every PPM row (top-down), the source row."""
    rows = row_map(H, row_block, world)
    maxrows = max(len(r) for r in rows)
    src = np.empty(H, np.int64)
    for r, jr in enumerate(rows):
        n = len(jr)
        k = np.arange(n)
        # local row k sits at position n-1-k; global row j is PPM row H-1-j
        src[H - 1 - jr] = r * maxrows + (n - 1 - k)
    return src, maxrows


class FrameGather:
    """Gathers per-rank RGB8 row buffers into the full PPM body on rank `dst` (one collective)."""

    def __init__(self, W, H, row_block, rank, world, device, dst=0, group=None):
        import torch
        self.W, self.H, self.rank, self.world, self.dst, self.group = W, H, rank, world, dst, group
        src, self.maxrows = ppm_row_permutation(H, row_block, world)
        self.local_rows = len(row_map(H, row_block, world)[rank])
        self.row_bytes = 3 * W
        # each rank renders into a padded buffer of maxrows rows; only the first local_rows are used
        self.local = torch.zeros((self.maxrows, self.row_bytes), dtype=torch.uint8, device=device)
        if rank == dst:
            self.recv = [torch.zeros_like(self.local) for _ in range(world)]
            self.perm = torch.as_tensor(src, device=device)
            self.full = torch.empty((H, self.row_bytes), dtype=torch.uint8, device=device)
        else:
            self.recv = None

    def local_ptr(self):
        return self.local.data_ptr()

    def gather(self):
        """Collective: returns the (H, 3W) PPM body on dst, None elsewhere (asynchronous on GPU)."""
        import torch
        import torch.distributed as dist
        if self.world == 1:
            return self.local[: self.H]
        dist.gather(self.local, self.recv if self.rank == self.dst else None, dst=self.dst, group=self.group)
        if self.rank != self.dst:
            return None
        stacked = torch.cat(self.recv, dim=0)
        torch.index_select(stacked, 0, self.perm, out=self.full)
        return self.full
