"""Framebuffer partitioning across GPUs and the RGB8 gather.

One process per GPU (torch.distributed; backend "nccl" = RCCL over xGMI on ROCm).  Rows are
dealt in blocks of `row_block` rows round-robin over ranks (block b -> rank b % world), which
balances the load: a mesh covers only the central rows of a frame, so contiguous bands
would leave most ranks idle.  A step renders a BATCH of F frames (e.g. the anim.cpp orbit):
every rank renders its rows of all F frames with ONE ceres_render_batch_device launch pair
into a compact RGB8 buffer (frame-major, local row k of a frame at position n - 1 - k), and
ONE collective per step -- a gather of those buffers to rank 0 -- brings all F frames there,
where ceres_assemble_rgb8 un-interleaves them into F PPM bodies (BatchGather), or -- the
bench's default, F = k N -- each frame is gathered to one owner rank (k frames per rank), all
those gathers as one all-to-all (FrameExchange), so no single rank's ingress carries the whole
step.  Both are
multi-buffered: the gather (RCCL stream) and assembly (side stream) of step k overlap the
render of step k + 1.  FrameOwner is the collective-free partition of the same step: each rank
renders its k frames whole (no row split, nothing to gather).  The scene is replicated (uploaded per device, outside the timed
region).  The reference has no distributed code (render.hpp:104 is an OpenMP loop).
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


def exchange_order(frames, world):
    """Batch order of an F-frame step for FrameExchange (F = k * world): batch frame q*k + m is
    orbit frame m*world + q, so rank q owns the consecutive batch frames q*k .. q*k+k-1 (orbit
    frames q, q + N, q + 2N, ...; batch frame 0 = orbit frame 0)."""
    k = frames // world
    return np.asarray([m * world + q for q in range(world) for m in range(k)], np.int64)


def band_height(H, world):
    """Rows per band of the band partition (FrameBands): ceil(H / world), rounded up to a multiple of
    the kernel's 8-row tiles when every band stays non-empty."""
    bh = -(-H // world)
    bh8 = -(-bh // 8) * 8
    return bh8 if (world - 1) * bh8 < H else bh


def band_rows(H, bh, b):
    """Rows of band b (the last band is shorter)."""
    return max(0, min(bh, H - b * bh))


def band_groups(frames, rank, world):
    """Batch frames whose band `b` this rank renders, per band: frame f's band on rank r is
    (r + f) mod world, so over the step's frames every rank renders every band equally often
    (a frame's cost is concentrated in its central bands; rotating keeps the ranks balanced)."""
    return [[f for f in range(frames) if (rank + f) % world == b] for b in range(world)]


def rank_rows(H, row_block, rank, world):
    """Closed form of len(row_map(...)[rank]) -- the formula ceres_assemble uses on the device."""
    nb = (H + row_block - 1) // row_block
    if rank >= nb:
        return 0
    mine = (nb - 1 - rank) // world + 1
    return mine * row_block - ((nb * row_block - H) if (nb - 1) % world == rank else 0)


def batch_row_permutation(H, row_block, world, frames):
    """For every output row (frame-major, PPM rows top-down), its row in the rank-major
    concatenation of the gathered buffers (each rank: `frames * maxrows` rows, its frames
    back to back with n_r rows each).  Returns (src [frames*H], maxrows)."""
    rows = row_map(H, row_block, world)
    maxrows = max(len(r) for r in rows)
    src = np.empty(frames * H, np.int64)
    for f in range(frames):
        for r, jr in enumerate(rows):
            n = len(jr)
            k = np.arange(n)
            # local row k of frame f sits at f*n + n-1-k; global row j is PPM row H-1-j
            src[f * H + H - 1 - jr] = r * frames * maxrows + f * n + (n - 1 - k)
    return src, maxrows


def ppm_row_permutation(H, row_block, world):
    """Single-frame batch_row_permutation (rank buffers of `maxrows` rows)."""
    return batch_row_permutation(H, row_block, world, 1)


class BatchGather:
    """Per-rank RGB8 buffers of an F-frame batch -> F PPM bodies on rank `dst`.

    slots: number of buffer sets (2 = double buffering: fill slot k%2 while slot (k-1)%2 is
    in flight).  On a GPU the un-interleave is ceres_assemble_rgb8 on a side stream; on CPU
    (gloo tests) it is the same permutation applied with index_select.
    """

    def __init__(self, W, H, row_block, rank, world, frames=1, device="cpu", dst=0, group=None, slots=2):
        import torch
        self.W, self.H, self.rank, self.world, self.dst, self.group = W, H, rank, world, dst, group
        self.frames, self.row_block, self.slots = frames, row_block, slots
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        src, self.maxrows = batch_row_permutation(H, row_block, world, frames)
        self.local_rows = rank_rows(H, row_block, rank, world)
        self.row_bytes = 3 * W
        rows = frames * self.maxrows
        # each rank's batch fills the first frames*local_rows rows; the rest pads to equal size
        self.bufs = [torch.zeros((rows, self.row_bytes), dtype=torch.uint8, device=self.device)
                     for _ in range(slots)]
        self.is_dst = rank == dst
        self.work = [None] * slots
        if self.is_dst and world > 1:
            self.recv = [torch.zeros((world, rows, self.row_bytes), dtype=torch.uint8, device=self.device)
                         for _ in range(slots)]
            self.full = [torch.empty((frames, H, self.row_bytes), dtype=torch.uint8, device=self.device)
                         for _ in range(slots)]
            self.perm = torch.as_tensor(src, device=self.device)
            if self.cuda:
                self.side = torch.cuda.Stream(device=self.device)
                self.assembled = [torch.cuda.Event() for _ in range(slots)]
                self.reused = [False] * slots

    def local_ptr(self, slot=0):
        return self.bufs[slot].data_ptr()

    def frame_view(self, slot=0):
        """World-1 output: the local buffer already is F PPM bodies."""
        return self.bufs[slot][: self.frames * self.H].view(self.frames, self.H, self.row_bytes)

    def start(self, slot=0):
        """Launch the gather of `slot` (call after the render into bufs[slot] is enqueued)."""
        import torch
        import torch.distributed as dist
        if self.world == 1:
            return
        if self.is_dst and self.cuda and self.reused[slot]:
            # recv[slot] must not be overwritten before the previous assembly read it
            torch.cuda.current_stream(self.device).wait_event(self.assembled[slot])
        recv = list(self.recv[slot].unbind(0)) if self.is_dst else None
        self.work[slot] = dist.gather(self.bufs[slot], recv, dst=self.dst, group=self.group, async_op=True)

    def finish(self, slot=0):
        """Complete `slot`: returns the (F, H, 3W) PPM bodies on dst (asynchronously, on the
        side stream for GPUs), None elsewhere.  Also makes local[slot] safe to overwrite."""
        import torch
        if self.world == 1:
            return self.frame_view(slot)
        w = self.work[slot]
        self.work[slot] = None
        if w is None:
            raise RuntimeError("BatchGather.finish without start")
        if not self.cuda:
            w.wait()
            if not self.is_dst:
                return None
            flat = self.recv[slot].view(-1, self.row_bytes)
            torch.index_select(flat, 0, self.perm, out=self.full[slot].view(-1, self.row_bytes))
            return self.full[slot]
        w.wait()                      # current stream: bufs[slot] may be reused after the send
        if not self.is_dst:
            return None
        import ceres_raytracer_amd as pkg
        with torch.cuda.stream(self.side):
            w.wait()                  # side stream waits for the collective
            pkg.assemble_rgb8(self.recv[slot].data_ptr(), self.recv[slot][0].numel(), self.full[slot].data_ptr(),
                              self.frames, self.W, self.H, self.row_block, self.world, self.side.cuda_stream)
            self.assembled[slot].record(self.side)
        self.reused[slot] = True
        return self.full[slot]

    def wait_assembled(self):
        """Make the current stream wait for every issued assembly (end of a timed region)."""
        import torch
        if self.is_dst and self.world > 1 and self.cuda:
            for s, used in enumerate(self.reused):
                if used:
                    torch.cuda.current_stream(self.device).wait_event(self.assembled[s])


def packed_row_permutation(H, row_block, world, frames):
    """batch_row_permutation for PACKED rank buffers (no padding: rank r's frames * n_r rows start
    right after rank r-1's) -- the receive layout of FrameExchange's all-to-all."""
    rows = row_map(H, row_block, world)
    off = np.cumsum([0] + [frames * len(r) for r in rows])
    src = np.empty(frames * H, np.int64)
    for f in range(frames):
        for r, jr in enumerate(rows):
            n = len(jr)
            k = np.arange(n)
            src[f * H + H - 1 - jr] = off[r] + f * n + (n - 1 - k)
    return src


class FrameExchange:
    """Per-rank RGB8 rows of an F-frame batch (F = k * world) -> frames [q*k, (q+1)*k) of the
    batch assembled on rank q.

    The weak-scaling step renders F frames, every frame's rows dealt over the N ranks;
    gathering all F frames to rank 0 would make rank 0's xGMI ingress (7 links) carry
    (N-1)/N of every frame of the step.  Instead each frame is gathered to ONE owner rank (the
    batch is ordered so that rank q owns the consecutive batch frames q*k .. q*k+k-1): all
    those gathers are one RCCL all-to-all (`all_to_all_single`, rank r's rows of rank q's
    frames -> rank q), each rank receives (N-1)/N of k frames over all its links, and
    un-interleaves them with ceres_assemble_rgb8_packed on a side stream.  Same slot protocol
    as BatchGather.
    """

    def __init__(self, W, H, row_block, rank, world, frames=None, device="cpu", group=None, slots=2):
        import torch
        frames = world if frames is None else frames
        if frames % world:
            raise ValueError("FrameExchange: frames (%d) must be a multiple of world (%d)" % (frames, world))
        self.W, self.H, self.rank, self.world, self.group = W, H, rank, world, group
        self.frames, self.row_block, self.slots = frames, row_block, slots
        self.k = frames // world                     # frames each rank assembles
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.rows = [rank_rows(H, row_block, r, world) for r in range(world)]
        self.local_rows = self.rows[rank]
        self.maxrows = max(self.rows)
        self.row_bytes = 3 * W
        self.bufs = [torch.zeros((frames * self.maxrows, self.row_bytes), dtype=torch.uint8, device=self.device)
                     for _ in range(slots)]
        self.work = [None] * slots
        self.is_dst = True                  # every rank assembles its k frames
        if world > 1:
            self.recv = [torch.zeros((self.k * H, self.row_bytes), dtype=torch.uint8, device=self.device)
                         for _ in range(slots)]
            self.full = [torch.empty((self.k, H, self.row_bytes), dtype=torch.uint8, device=self.device)
                         for _ in range(slots)]
            self.perm = torch.as_tensor(packed_row_permutation(H, row_block, world, self.k), device=self.device)
            self.in_splits = [self.k * self.local_rows * self.row_bytes] * world
            self.out_splits = [self.k * n * self.row_bytes for n in self.rows]
            if self.cuda:
                self.side = torch.cuda.Stream(device=self.device)
                self.assembled = [torch.cuda.Event() for _ in range(slots)]
                self.reused = [False] * slots

    def owned_frames(self):
        """Batch frame indices this rank assembles (in the order finish() returns them)."""
        return list(range(self.rank * self.k, (self.rank + 1) * self.k))

    def local_ptr(self, slot=0):
        return self.bufs[slot].data_ptr()

    def frame_view(self, slot=0):
        return self.bufs[slot][: self.frames * self.H].view(self.frames, self.H, self.row_bytes)

    def start(self, slot=0):
        import torch
        import torch.distributed as dist
        if self.world == 1:
            return
        if self.cuda and self.reused[slot]:
            torch.cuda.current_stream(self.device).wait_event(self.assembled[slot])
        send = self.bufs[slot][: self.frames * self.local_rows].view(-1)
        self.work[slot] = dist.all_to_all_single(self.recv[slot].view(-1), send, self.out_splits, self.in_splits,
                                                 group=self.group, async_op=True)

    def finish(self, slot=0):
        """Complete `slot`: returns this rank's k frames (batch frames owned_frames()) as
        (k, H, 3W) PPM bodies (asynchronously, on the side stream for GPUs)."""
        import torch
        if self.world == 1:
            return self.frame_view(slot)
        w = self.work[slot]
        self.work[slot] = None
        if w is None:
            raise RuntimeError("FrameExchange.finish without start")
        w.wait()
        if not self.cuda:
            torch.index_select(self.recv[slot], 0, self.perm, out=self.full[slot].view(-1, self.row_bytes))
            return self.full[slot]
        import ceres_raytracer_amd as pkg
        with torch.cuda.stream(self.side):
            w.wait()
            pkg.assemble_rgb8_packed(self.recv[slot].data_ptr(), self.full[slot].data_ptr(), self.k, self.W, self.H,
                                     self.row_block, self.world, self.side.cuda_stream)
            self.assembled[slot].record(self.side)
        self.reused[slot] = True
        return self.full[slot]

    def wait_assembled(self):
        import torch
        if self.world > 1 and self.cuda:
            for s, used in enumerate(self.reused):
                if used:
                    torch.cuda.current_stream(self.device).wait_event(self.assembled[s])


class FrameBands:
    """Per-rank bands of an F-frame batch (F = k * world) -> frames [q*k, (q+1)*k) of the batch
    assembled on rank q, with nothing to un-interleave.

    The renders use ceres_tiling.bands (Tiling(band_height, rank, world, bands=1)): frame f of the
    batch is cut into `world` contiguous bands and rank r renders band (r + f) mod world, so over
    the step's frames every rank renders every band equally often (the frames' cost sits in their
    central bands).  A rank's buffer holds its band of every frame, frame-major, `band_height` rows
    per frame with the band's valid rows at the END (ceres_tiling: positions row_block - n .. of the
    frame, top row first) -- a contiguous slice of the frame's PPM body.  start() sends each band
    to the frame's owner and receives the owner's bands straight into their rows of its PPM
    bodies: point-to-point RCCL (batch_isend_irecv; one message per (frame, peer)), no staging
    buffer and no assembly kernel (FrameExchange un-interleaves row blocks after its all-to-all,
    which costs ~9 % of an N = 8 step in the one-GPU rehearsal).  Own bands are copied locally.
    Same slot protocol as FrameExchange.
    """

    def __init__(self, W, H, rank, world, frames=None, device="cpu", group=None, slots=2):
        import torch
        frames = world if frames is None else frames
        if frames % world:
            raise ValueError("FrameBands: frames (%d) must be a multiple of world (%d)" % (frames, world))
        self.W, self.H, self.rank, self.world, self.group = W, H, rank, world, group
        self.frames, self.slots = frames, slots
        self.k = frames // world
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.band = band_height(H, world) if world > 1 else H
        self.local_rows = self.band                  # every frame: one band (ceres_tiling_local_rows)
        self.row_bytes = 3 * W
        self.is_dst = True
        self.bufs = [torch.zeros((frames * self.band, self.row_bytes), dtype=torch.uint8, device=self.device)
                     for _ in range(slots)]
        self.full = [torch.zeros((self.k, H, self.row_bytes), dtype=torch.uint8, device=self.device)
                     for _ in range(slots)] if world > 1 else None
        self.work = [None] * slots

    def tiling_args(self):
        """(row_block, rank, world, bands) of this rank's renders."""
        return (self.band, self.rank, self.world, 1 if self.world > 1 else 0)

    def owned_frames(self):
        return list(range(self.rank * self.k, (self.rank + 1) * self.k))

    def local_ptr(self, slot=0):
        return self.bufs[slot].data_ptr()

    def _band_view(self, slot, f):
        """This rank's band of batch frame f in its buffer (the band's valid rows only)."""
        b = (self.rank + f) % self.world
        n = band_rows(self.H, self.band, b)
        return self.bufs[slot][f * self.band + self.band - n:(f + 1) * self.band], b, n

    def _frame_slice(self, slot, m, b):
        """Rows of band b in owned frame m's PPM body (top row first: band b's global rows
        b*band .. b*band + n - 1 are PPM rows H - b*band - n .. H - b*band - 1)."""
        n = band_rows(self.H, self.band, b)
        top = self.H - b * self.band - n
        return self.full[slot][m, top:top + n]

    def start(self, slot=0):
        import torch.distributed as dist
        if self.world == 1:
            return
        ops = []
        for m, f in enumerate(self.owned_frames()):  # own bands of own frames: local copies
            src, b, n = self._band_view(slot, f)
            if n:
                self._frame_slice(slot, m, b).copy_(src)
        for q in range(self.world):                 # this rank's bands of q's frames -> q
            if q == self.rank:
                continue
            for f in range(q * self.k, (q + 1) * self.k):
                src, b, n = self._band_view(slot, f)
                if n:
                    ops.append(dist.P2POp(dist.isend, src.view(-1), q, group=self.group))
        for r in range(self.world):                 # r's bands of this rank's frames, in place
            if r == self.rank:
                continue
            for m, f in enumerate(self.owned_frames()):
                b = (r + f) % self.world
                if band_rows(self.H, self.band, b):
                    ops.append(dist.P2POp(dist.irecv, self._frame_slice(slot, m, b).view(-1), r, group=self.group))
        self.work[slot] = dist.batch_isend_irecv(ops) if ops else []

    def finish(self, slot=0):
        """Complete `slot`: this rank's k frames (batch frames owned_frames()) as (k, H, 3W) PPM
        bodies (for GPUs: ordered on the current stream)."""
        if self.world == 1:
            return self.bufs[slot][: self.frames * self.H].view(self.frames, self.H, self.row_bytes)
        w = self.work[slot]
        self.work[slot] = None
        if w is None:
            raise RuntimeError("FrameBands.finish without start")
        for x in w:
            x.wait()
        return self.full[slot]

    def wait_assembled(self):
        pass


class FrameOwner:
    """Unsplit frames (no collective): rank q renders its k = F/N frames of the step WHOLE, straight
    into PPM bodies in its own HBM -- batch frames q*k .. q*k+k-1 of exchange_order, i.e. orbit
    frames q, q + N, q + 2N, ..., so every rank samples the whole orbit and the ranks' loads stay
    balanced.  Frames are independent (render.hpp:104-153 touches one frame's pixels), so the step
    has no data-path exchange at all: the xGMI links carry nothing, and a rank's work is k whole
    frames at every N.  Same interface as FrameExchange (start/finish/wait_assembled are no-ops
    beyond handing back the rank's own buffer).
    """

    def __init__(self, W, H, rank, world, frames=None, device="cpu", slots=2):
        import torch
        frames = world if frames is None else frames
        if frames % world:
            raise ValueError("FrameOwner: frames (%d) must be a multiple of world (%d)" % (frames, world))
        self.W, self.H, self.rank, self.world = W, H, rank, world
        self.frames, self.slots = frames, slots
        self.k = frames // world
        self.device = torch.device(device)
        self.local_rows = H                  # whole frames
        self.row_bytes = 3 * W
        self.is_dst = True
        self.bufs = [torch.zeros((self.k * H, self.row_bytes), dtype=torch.uint8, device=self.device)
                     for _ in range(slots)]

    def owned_frames(self):
        """Batch frame indices (exchange_order) this rank renders, in buffer order."""
        return list(range(self.rank * self.k, (self.rank + 1) * self.k))

    def local_ptr(self, slot=0):
        return self.bufs[slot].data_ptr()

    def frame_view(self, slot=0):
        return self.bufs[slot].view(self.k, self.H, self.row_bytes)

    def start(self, slot=0):
        return None

    def finish(self, slot=0):
        return self.frame_view(slot)

    def wait_assembled(self):
        return None


class FrameGather(BatchGather):
    """Single frame, single buffer: gather() = start() + finish() -> (H, 3W) PPM body on dst."""

    def __init__(self, W, H, row_block, rank, world, device, dst=0, group=None):
        super().__init__(W, H, row_block, rank, world, frames=1, device=device, dst=dst, group=group, slots=1)
        self.local = self.bufs[0]          # (maxrows, 3W): local row k at position local_rows-1-k

    def gather(self):
        self.start(0)
        out = self.finish(0)
        if out is None:
            return None
        if self.cuda and self.is_dst and self.world > 1:
            import torch
            torch.cuda.current_stream(self.device).wait_event(self.assembled[0])
        return out[0]
