"""Multi-rank framebuffer partition + gather on CPU with the gloo backend.

Each rank fills its local RGB8 buffer exactly as ceres_render_device lays it out (its rows of
the reference PPM -- from the golden fixture -- local row k at position n-1-k), then
FrameGather assembles the frame on rank 0 with one collective; the result must be the
reference PPM byte for byte.  The GPU side of the same path is tests/test_gpu_parity.py.
"""
import gzip
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN, REPO, import_package


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, name, W, H, row_block, q):
    import sys
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from conftest import import_package as ip
    pkg = ip()
    import ceres_raytracer_amd.distributed as D
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        with open(os.path.join(GOLDEN, name + ".exact.ppm.gz"), "rb") as f:
            ppm = gzip.decompress(f.read())
        hdr = len(b"P6 %d %d 255\n" % (W, H))
        body = np.frombuffer(ppm[hdr:], np.uint8).reshape(H, 3 * W)
        g = D.FrameGather(W, H, row_block, rank, world, device="cpu")
        rows = D.row_map(H, row_block, world)[rank]
        assert g.local_rows == len(rows) == pkg.local_rows(H, pkg.Tiling(row_block, rank, world))
        n = len(rows)
        for k, j in enumerate(rows):
            g.local[n - 1 - k] = torch.from_numpy(body[H - 1 - j].copy())
        full = g.gather()
        if rank == 0:
            q.put(bool(np.array_equal(full.numpy(), body)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,row_block", [(2, 16), (3, 7), (2, 1000)])
def test_gather_reassembles_reference_frame(world, row_block):
    import_package()
    name, W, H = "dragon_333x217", 333, 217
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, W, H, row_block, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert q.get(timeout=10) is True


def _batch_worker(rank, world, port, W, H, row_block, frames, q, slots=2):
    import sys
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from conftest import import_package as ip
    ip()
    import ceres_raytracer_amd.distributed as D
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        bodies = []
        for name in ("dragon_333x217", "dragon_orbit3_333x217"):
            with open(os.path.join(GOLDEN, name + ".exact.ppm.gz"), "rb") as f:
                ppm = gzip.decompress(f.read())
            hdr = len(b"P6 %d %d 255\n" % (W, H))
            bodies.append(np.frombuffer(ppm[hdr:], np.uint8).reshape(H, 3 * W))
        rng = np.random.default_rng(7)
        steps = 3 * slots                          # bench.py's rotation: step k uses slot k % slots
        while len(bodies) < steps * frames:
            bodies.append(rng.integers(0, 256, size=(H, 3 * W), dtype=np.uint8))
        g = D.BatchGather(W, H, row_block, rank, world, frames=frames, device="cpu", slots=slots)
        rows = D.row_map(H, row_block, world)[rank]
        n = len(rows)
        assert g.local_rows == n
        ok = True
        owner = [None] * slots                     # step whose batch a slot holds in flight

        def check(slot):
            nonlocal ok
            full = g.finish(slot)
            k = owner[slot]
            if rank == 0:
                for f in range(frames):
                    ok &= bool(np.array_equal(full[f].numpy(), bodies[k * frames + f]))
            else:
                ok &= full is None
            owner[slot] = None

        for k in range(steps):                     # up to `slots` steps in flight
            slot = k % slots
            if owner[slot] is not None:
                check(slot)
            for f in range(frames):
                body = bodies[k * frames + f]
                for i, j in enumerate(rows):
                    g.bufs[slot][f * n + n - 1 - i] = torch.from_numpy(body[H - 1 - j].copy())
            g.start(slot)
            owner[slot] = k
        for slot in range(slots):
            if owner[slot] is not None:
                check(slot)
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,row_block,frames,slots", [(2, 16, 2, 2), (3, 7, 3, 2), (4, 16, 4, 2), (2, 8, 2, 4),
                                                           (3, 8, 3, 4)])
def test_batch_gather_double_buffered(world, row_block, frames, slots):
    """F-frame batches (the bench's weak-scaling step), `slots` steps in flight rotating as in
    bench.py (the step-stream rotation), gloo on CPU."""
    import_package()
    W, H = 333, 217
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_batch_worker, args=(r, world, port, W, H, row_block, frames, q, slots))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
        assert p.exitcode == 0
    res = dict(q.get(timeout=10) for _ in range(world))
    assert all(res.values()), res


def test_rank_rows_closed_form():
    import_package()
    import ceres_raytracer_amd.distributed as D
    for H in (1, 7, 16, 17, 217, 1080, 4096):
        for world in (1, 2, 3, 5, 8):
            for rb in (1, 5, 16, 1000):
                for r in range(world):
                    assert D.rank_rows(H, rb, r, world) == len(D.row_map(H, rb, world)[r])


def test_row_map_covers_every_row_once():
    pkg = import_package()
    import ceres_raytracer_amd.distributed as D
    for H in (1, 15, 16, 17, 1080, 4096):
        for world in (1, 2, 3, 8):
            for rb in (1, 16, 64):
                rows = D.row_map(H, rb, world)
                allr = np.sort(np.concatenate(rows))
                np.testing.assert_array_equal(allr, np.arange(H))
                for r in range(world):
                    assert len(rows[r]) == pkg.local_rows(H, pkg.Tiling(rb, r, world))


def _exchange_worker(rank, world, port, W, H, row_block, slots, q, k=1):
    import sys
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from conftest import import_package as ip
    ip()
    import torch
    import torch.distributed as dist
    import ceres_raytracer_amd.distributed as D
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(11)
        steps = 3 * slots
        F = k * world
        bodies = [rng.integers(0, 256, size=(H, 3 * W), dtype=np.uint8) for _ in range(steps * F)]
        g = D.FrameExchange(W, H, row_block, rank, world, frames=F, device="cpu", slots=slots)
        assert g.owned_frames() == list(range(rank * k, rank * k + k))
        rows = D.row_map(H, row_block, world)[rank]
        n = len(rows)
        assert g.local_rows == n
        ok = True
        owner = [None] * slots

        def check(slot):
            nonlocal ok
            full = g.finish(slot)
            st = owner[slot]
            for m, f in enumerate(g.owned_frames()):  # batch frames rank*k .. rank*k + k - 1
                ok &= bool(np.array_equal(full[m].numpy(), bodies[st * F + f]))
            owner[slot] = None

        for st in range(steps):
            slot = st % slots
            if owner[slot] is not None:
                check(slot)
            for f in range(F):                       # frame-major, compact (n rows per frame)
                body = bodies[st * F + f]
                for i, j in enumerate(rows):
                    g.bufs[slot][f * n + n - 1 - i] = torch.from_numpy(body[H - 1 - j].copy())
            g.start(slot)
            owner[slot] = st
        for slot in range(slots):
            if owner[slot] is not None:
                check(slot)
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,row_block,slots,k", [(2, 16, 2, 1), (3, 7, 4, 1), (4, 8, 2, 4), (5, 3, 3, 2),
                                                     (2, 8, 4, 4), (8, 8, 8, 16)])
def test_frame_exchange_alltoall(world, row_block, slots, k):
    """bench.py's default N > 1 collective: each of the step's k*N frames is gathered to its owner
    rank (one all-to-all; rank q owns batch frames q*k .. q*k+k-1), `slots` steps in flight,
    gloo on CPU; ragged row counts per rank.  (8, 8, 8, 16) is the driver's N = 8 bench shape:
    8-row blocks, 8 step slots, 16 owned frames per rank (128 per step), on small frames."""
    import_package()
    W, H = 97, 61
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exchange_worker, args=(r, world, port, W, H, row_block, slots, q, k)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
        assert p.exitcode == 0
    res = dict(q.get(timeout=10) for _ in range(world))
    assert all(res.values()), res


def test_band_geometry():
    """ceres_tiling.bands: world contiguous bands of band_height rows (multiple of the 8-row tile
    when every band stays non-empty) cover every row once; the library's local row count is the
    band height; over a step every rank renders every band equally often (band_groups)."""
    pkg = import_package()
    import ceres_raytracer_amd.distributed as D
    for H in (1, 7, 15, 16, 61, 217, 1080, 2160, 4096):
        for world in (2, 3, 4, 5, 8):
            if world > H:
                continue
            bh = D.band_height(H, world)
            rows = [D.band_rows(H, bh, b) for b in range(world)]
            assert sum(rows) == H, (H, world, bh, rows)
            # bands are non-empty unless the frame is too short to give every rank a row of ceil(H / N)
            assert all(n > 0 for n in rows) or (world - 1) * -(-H // world) >= H, (H, world, rows)
            assert bh * world >= H and (bh % 8 == 0 or (world - 1) * (-(-bh // 8) * 8) >= H)
            for r in range(world):
                assert pkg.local_rows(H, pkg.Tiling(bh, r, world, 1)) == bh
    for world, k in ((2, 16), (8, 16), (3, 2)):
        for r in range(world):
            g = D.band_groups(k * world, r, world)
            assert [len(x) for x in g] == [k] * world
            assert sorted(f for x in g for f in x) == list(range(k * world))
    assert D.band_height(1080, 8) == 136 and D.band_rows(1080, 136, 7) == 128


def _bands_worker(rank, world, port, W, H, slots, q, k):
    import sys
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from conftest import import_package as ip
    ip()
    import torch
    import torch.distributed as dist
    import ceres_raytracer_amd.distributed as D
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(23)
        steps = 3 * slots
        F = k * world
        bodies = [rng.integers(0, 256, size=(H, 3 * W), dtype=np.uint8) for _ in range(steps * F)]
        g = D.FrameBands(W, H, rank, world, frames=F, device="cpu", slots=slots)
        assert g.owned_frames() == list(range(rank * k, rank * k + k))
        bh = g.band
        assert g.local_rows == bh and g.tiling_args() == (bh, rank, world, 1)
        ok = True
        owner = [None] * slots

        def check(slot):
            nonlocal ok
            full = g.finish(slot)
            st = owner[slot]
            for m, f in enumerate(g.owned_frames()):
                ok &= bool(np.array_equal(full[m].numpy(), bodies[st * F + f]))
            owner[slot] = None

        for st in range(steps):
            slot = st % slots
            if owner[slot] is not None:
                check(slot)
            g.bufs[slot].fill_(0)
            for f in range(F):                       # as the kernel writes RGB8 with ceres_tiling.bands
                b = (rank + f) % world
                for i in range(D.band_rows(H, bh, b)):   # local row i = global row b*bh + i at position bh-1-i
                    j = b * bh + i
                    g.bufs[slot][f * bh + bh - 1 - i] = torch.from_numpy(bodies[st * F + f][H - 1 - j].copy())
            g.start(slot)
            owner[slot] = st
        for slot in range(slots):
            if owner[slot] is not None:
                check(slot)
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,slots,k,H", [(2, 2, 1, 61), (3, 3, 2, 61), (4, 2, 4, 97), (5, 4, 2, 33), (8, 8, 16, 61)])
def test_frame_bands_p2p(world, slots, k, H):
    """bench.py --collect bands: each rank renders band (rank + f) mod N of every frame f and the
    bands travel point to point into their owner's PPM bodies (no un-interleave), `slots` steps in
    flight, gloo on CPU; ragged last bands.  (8, 8, 16) is the N = 8 bench shape (128 frames per
    step, 16 owned per rank) on small frames."""
    import_package()
    W = 13
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bands_worker, args=(r, world, port, W, H, slots, q, k)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
        assert p.exitcode == 0
    res = dict(q.get(timeout=10) for _ in range(world))
    assert all(res.values()), res


def test_packed_permutation_matches_padded():
    """packed_row_permutation = batch_row_permutation with the padding rows squeezed out."""
    import_package()
    import ceres_raytracer_amd.distributed as D
    for H, rb, world, frames in [(61, 3, 5, 1), (217, 16, 4, 3), (1080, 8, 8, 1)]:
        rows = D.row_map(H, rb, world)
        maxrows = max(len(r) for r in rows)
        padded, _ = D.batch_row_permutation(H, rb, world, frames)
        packed = D.packed_row_permutation(H, rb, world, frames)
        off = np.cumsum([0] + [frames * len(r) for r in rows])
        r_of = padded // (frames * maxrows)
        np.testing.assert_array_equal(packed, off[r_of] + padded % (frames * maxrows))


@pytest.mark.parametrize("world,k", [(1, 16), (2, 16), (3, 2), (4, 16), (8, 16), (8, 1)])
def test_frame_owner_partition(world, k):
    """bench.py --collect frames (the default except for tiled C4/C5 at N != 2): rank q renders
    batch frames q*k .. q*k+k-1 of exchange_order WHOLE -- orbit frames q, q+N, q+2N, ... -- so
    the ranks' frames partition the step, each rank samples the whole orbit (consecutive frames
    of a rank are N orbit frames apart), and the rank's buffer already holds its k PPM bodies
    (finish() hands back the buffer itself: no collective, no copy)."""
    import_package()
    import ceres_raytracer_amd.distributed as D
    W, H = 13, 7
    F = k * world
    order = D.exchange_order(F, world)
    seen = []
    for q in range(world):
        g = D.FrameOwner(W, H, q, world, frames=F, device="cpu", slots=2)
        assert g.local_rows == H and g.k == k
        own = g.owned_frames()
        orbit = [int(order[f]) for f in own]
        assert orbit == [q + m * world for m in range(k)]
        seen += orbit
        assert tuple(g.bufs[1].shape) == (k * H, 3 * W)
        assert g.start(1) is None
        out = g.finish(1)
        assert tuple(out.shape) == (k, H, 3 * W) and out.data_ptr() == g.bufs[1].data_ptr()
    assert sorted(seen) == list(range(F))
    with pytest.raises(ValueError):
        D.FrameOwner(W, H, 0, world + 1, frames=(world + 1) * k + 1)


def _owner_worker(rank, world, port, W, H, k, q):
    import sys
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from conftest import import_package as ip
    ip()
    import hashlib
    import torch
    import torch.distributed as dist
    import ceres_raytracer_amd.distributed as D
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        F = k * world
        order = D.exchange_order(F, world)
        ok = True
        g = D.FrameOwner(W, H, rank, world, frames=F, device="cpu", slots=2)

        def body(orbit_f, step):                    # the frame a renderer would produce for this view
            rng = np.random.default_rng(1000 * step + orbit_f)
            return rng.integers(0, 256, size=(H, 3 * W), dtype=np.uint8)

        for step in range(4):                        # bench.py's protocol: render into the slot, start, finish
            slot = step % 2
            for m, f in enumerate(g.owned_frames()):
                g.bufs[slot][m * H:(m + 1) * H] = torch.from_numpy(body(int(order[f]), step))
            g.start(slot)
            full = g.finish(slot)
            g.wait_assembled()
            # validation as bench.py does it: every rank checks its own frames, then one all_reduce
            got = torch.zeros(F, dtype=torch.int64)
            for m, f in enumerate(g.owned_frames()):
                h = hashlib.sha256(full[m].numpy().tobytes()).hexdigest()
                got[int(order[f])] += int(h == hashlib.sha256(body(int(order[f]), step).tobytes()).hexdigest())
            dist.all_reduce(got)
            ok &= bool((got == 1).all())
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,k", [(2, 16), (4, 3)])
def test_frame_owner_gloo_step(world, k):
    """The collective-free partition through bench.py's step protocol on `world` gloo ranks: every
    orbit frame of every step is produced by exactly one rank and checked there (all_reduce of the
    per-frame matches = 1 for every frame)."""
    import_package()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_owner_worker, args=(r, world, port, 17, 9, k, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
        assert p.exitcode == 0
    res = dict(q.get(timeout=10) for _ in range(world))
    assert all(res.values()), res


def test_bench_partition_choice():
    """bench.py --collect auto: whole frames per rank with no data-path collective for the
    frame-unit configs (C3, bunny) at every N > 1; the tiled 4096^2 / 4K configs (C4, C5) cut their
    frames into rotated contiguous bands sent point to point to the owner ranks at N >= 4, and
    render whole frames at N = 2 (one xGMI link, DESIGN.md "Multi-GPU"); explicit choices are kept;
    a frame count that is not a multiple of N falls back to the gather.  The other partition is
    reported beside it (`alt_collect`)."""
    import sys
    sys.path.insert(0, REPO)
    import bench
    import configs
    C = configs.CONFIGS
    for n in (2, 4, 8):
        assert bench.choose_collect("auto", C["dragon_1080"], n, 16 * n) == "frames"
        assert bench.choose_collect("auto", C["bunny_1080"], n, 16 * n) == "frames"
    for name in ("dragon_4096", "proc_c5"):
        assert bench.choose_collect("auto", C[name], 2, 32) == "frames"
        assert bench.choose_collect("auto", C[name], 4, 64) == "bands"
        assert bench.choose_collect("auto", C[name], 8, 128) == "bands"
    assert bench.choose_collect("exchange", C["dragon_1080"], 4, 64) == "exchange"
    assert bench.choose_collect("bands", C["dragon_1080"], 4, 64) == "bands"
    assert bench.choose_collect("gather", C["dragon_1080"], 4, 64) == "gather"
    assert bench.choose_collect("frames", C["dragon_1080"], 3, 16) == "gather"
    assert bench.choose_collect("bands", C["dragon_1080"], 3, 16) == "gather"
    assert bench.alt_collect("bands") == "frames" and bench.alt_collect("frames") == "bands"
    assert bench.alt_collect("exchange") == "frames"


def _line_worker(rank, world, port, q):
    """Both partitions of a bench step through the slot protocol on gloo, then bench.py's result
    line built on rank 0 from the ranks' max wall time (as bench.py does at N > 1)."""
    import sys
    import time
    sys.path.insert(0, os.path.join(REPO, "tests"))
    sys.path.insert(0, REPO)
    from conftest import import_package as ip
    ip()
    import hashlib
    import bench
    import configs
    import ceres_raytracer_amd.distributed as D
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg = dict(configs.CONFIGS["dragon_1080"], W=17, H=23)      # the C3 config at a tiny size
        W, H, k, rb = cfg["W"], cfg["H"], 3, 4
        F = k * world
        order = D.exchange_order(F, world)
        collect = bench.choose_collect("auto", cfg, world, F)
        res = {}
        for col in (collect, bench.alt_collect(collect)):
            g = (D.FrameOwner(W, H, rank, world, frames=F, device="cpu", slots=2) if col == "frames" else
                 D.FrameBands(W, H, rank, world, frames=F, device="cpu", slots=2) if col == "bands" else
                 D.FrameExchange(W, H, rb, rank, world, frames=F, device="cpu", slots=2))
            rows = D.row_map(H, rb, world)[rank] if col == "exchange" else np.arange(H)

            def body(orbit_f, step):
                rng = np.random.default_rng(1000 * step + orbit_f)
                return rng.integers(0, 256, size=(H, 3 * W), dtype=np.uint8)

            ok = True
            t0 = time.perf_counter()
            for step in range(4):
                slot = step % 2
                if col == "frames":
                    for m, f in enumerate(g.owned_frames()):
                        g.bufs[slot][m * H:(m + 1) * H] = torch.from_numpy(body(int(order[f]), step))
                elif col == "bands":                     # band (rank + f) mod N of every frame, ceres_tiling.bands
                    bh = g.band
                    for f in range(F):
                        b = body(int(order[f]), step)
                        band = (rank + f) % world
                        for kk in range(D.band_rows(H, bh, band)):
                            g.bufs[slot][f * bh + bh - 1 - kk] = torch.from_numpy(b[H - 1 - (band * bh + kk)].copy())
                else:                                    # this rank's rows of every frame, ceres_tiling layout
                    n = len(rows)
                    for f in range(F):
                        b = body(int(order[f]), step)
                        for kk, j in enumerate(rows):
                            g.bufs[slot][f * n + n - 1 - kk] = torch.from_numpy(b[H - 1 - j].copy())
                g.start(slot)
                full = g.finish(slot)
                g.wait_assembled()
                got = torch.zeros(F, dtype=torch.int64)
                for m, f in enumerate(g.owned_frames()):
                    h = hashlib.sha256(full[m].numpy().tobytes()).hexdigest()
                    got[int(order[f])] += int(h == hashlib.sha256(body(int(order[f]), step).tobytes()).hexdigest())
                dist.all_reduce(got)
                ok &= bool((got == 1).all())
            el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
            dist.all_reduce(el, op=dist.ReduceOp.MAX)
            res[col] = (ok, float(el.item()))
        if rank == 0:
            rays = F * W * H + 100
            alt_c = bench.alt_collect(collect)
            alt = {"collect": alt_c, "value": round(rays * 4 / res[alt_c][1] / 1e6, 3)}
            line = bench.result_line(config_name="dragon_1080", cfg=cfg, world=dist.get_world_size(),
                                     backend=dist.get_backend(), collect=collect, views_kind="config", F=F, steps=4,
                                     warmup=0, T=res[collect][1], rays_step=rays, hits_step=50, full_mode=True,
                                     row_block=rb, streams=2, float_fb=False, arith="fma", roofline=None,
                                     roofline_step=None, roofline_solo=None, cpu=None, parity=None, alt=alt)
            q.put((all(v[0] for v in res.values()), json_dumps(line)))
    finally:
        dist.destroy_process_group()


def json_dumps(x):
    import json
    return json.dumps(x)


def test_bench_line_world2_gloo():
    """bench.py's N > 1 path on two gloo ranks: the headline partition for C3 is the collective-free
    `frames` partition (each rank's frames whole), the framebuffer exchange (rows over the ranks +
    one all-to-all) is run as `partition_alt`, every frame of both is produced exactly once, and the
    line names the world size and backend the collectives ran with."""
    import json
    import_package()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_line_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
        assert p.exitcode == 0
    ok, line = q.get(timeout=10)
    line = json.loads(line)
    assert ok
    assert line["n_gpus"] == line["world_size"] == 2 and line["backend"] == "gloo"
    assert line["config"]["collect"] == "frames"
    assert line["config"]["views"] == "config" and "copies of the config view" in line["config"]["workload"]
    assert line["partition_alt"]["collect"] == "bands" and line["partition_alt"]["value"] > 0
    assert line["scaling"] == "weak" and line["value"] > 0
