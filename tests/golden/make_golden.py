#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the REFERENCE's own hot path.

Runs oracle/_ref/ref_render (reference CMake flags, CMakeLists.txt:11-13) and
oracle/_ref/ref_render_exact (same + -ffp-contract=off) -- both compiled by oracle/Makefile
from the unmodified headers in /root/reference through oracle/ref_harness.cpp -- on every
config in ceres-raytracer_amd/configs.py and commits only small artefacts:

  <cfg>.json            rays/hits (render.hpp:155), node-pair / triangle-test statistics
                        (single_ray_traverser.hpp:132-135), camera basis as hex floats
                        (render.hpp:91-97), sha256 of the PPM (static.cpp:135-147) for both
                        contraction modes, sha256 of the rotated Triangle[] / tri_norms[]
                        bits and of the canonical (DFS) BVH topology, differing PPM bytes
                        between the two modes
  <cfg>.exact.ppm.gz    PPM of the contraction-free build   (configs <= 640x480 only)
  <cfg>.ref.ppm.gz      PPM of the reference-flag build     (only where it differs)
  <cfg>.records.npz     per-pixel {pixel, prim, t, u, v, shadow, rgb} of the contraction-free
                        build, every pixel for small configs, a seeded sample otherwise
  <cfg>.ref.records.npz the same for the reference-flag build; its scene hashes, camera basis,
                        pose and statistics are the "ref*" keys of <cfg>.json

Must run in the build container (needs /root/reference); the GPU box only reads the outputs.
Usage: python tests/golden/make_golden.py [cfg ...]
       python tests/golden/make_golden.py --orbit cfg ...   (orbit/<cfg>.json: every bench view)
"""
import gzip
import hashlib
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "ceres-raytracer_amd"))
import configs  # noqa: E402

REF = os.path.join(REPO, "oracle", "_ref", "ref_render")
REF_EXACT = os.path.join(REPO, "oracle", "_ref", "ref_render_exact")
SCRATCH = os.path.join(REPO, ".scratch", "golden")
SMALL = 640 * 480
SAMPLE_HITS, SAMPLE_OTHER, SEED = 4096, 1024, 12345

REC_DTYPE = np.dtype([("i", "<u4"), ("j", "<u4"), ("prim", "<i4"), ("t", "<f4"), ("u", "<f4"), ("v", "<f4"),
                      ("shadow", "<i4"), ("r", "<f4"), ("g", "<f4"), ("b", "<f4")])


def sha(path_or_bytes):
    h = hashlib.sha256()
    if isinstance(path_or_bytes, (bytes, bytearray)):
        h.update(path_or_bytes)
    else:
        with open(path_or_bytes, "rb") as f:
            for chunk in iter(lambda: f.read(1 << 22), b""):
                h.update(chunk)
    return h.hexdigest()


def canonical_bvh_sha(nodes32: bytes, prim64: bytes) -> str:
    """sha256 of the BVH topology in DFS order, independent of node numbering.

    Per node (bvh.hpp:25-79): 6 bound floats, primitive_count; leaves append their
    primitive_indices[first:first+count] (original triangle ids); inner nodes recurse
    into first_child then first_child + 1 (children are adjacent, bvh.hpp:9-13).
    """
    nodes = np.frombuffer(nodes32, dtype=np.uint32).reshape(-1, 8)
    prim = np.frombuffer(prim64, dtype=np.uint64)
    h = hashlib.sha256()
    stack = [0]
    while stack:
        k = stack.pop()
        n = nodes[k]
        h.update(n[:7].tobytes())
        cnt, first = int(n[6]), int(n[7])
        if cnt:
            h.update(prim[first:first + cnt].tobytes())
        else:
            stack.append(first + 1)
            stack.append(first)
    return h.hexdigest()


def run(binary, cfg, extra):
    cmd = [binary] + configs.cli_args(cfg) + extra
    out = subprocess.run(cmd, check=True, capture_output=True, text=True).stdout
    return json.loads(out.strip().splitlines()[-1])


def _sample(rec, small):
    if small:
        return np.arange(rec.size)
    rng = np.random.default_rng(SEED)
    hit = np.flatnonzero(rec["prim"] >= 0)
    other = np.flatnonzero(rec["prim"] < 0)
    return np.sort(np.concatenate([rng.choice(hit, min(SAMPLE_HITS, hit.size), replace=False),
                                   rng.choice(other, min(SAMPLE_OTHER, other.size), replace=False)]))


def _save_records(path, rec, keep, W):
    r = rec[keep]
    np.savez_compressed(path, pixel=(r["j"].astype(np.uint64) * W + r["i"]).astype(np.uint32),
                        prim=r["prim"], t=r["t"], u=r["u"], v=r["v"], shadow=r["shadow"],
                        rgb=np.stack([r["r"], r["g"], r["b"]], axis=1))


def _scene_hashes(p_dump):
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    nodes = np.fromfile(p_dump + ".nodes32", dtype=np.uint32)
    prim = np.fromfile(p_dump + ".prim64", dtype=np.uint64)
    return {"tri48_sha256": sha(p_dump + ".tri48"), "norm36_sha256": sha(p_dump + ".norm36"),
            "bvh_canonical_sha256": oracle.canonical_bvh_sha(nodes, prim)}


STAT_KEYS = ("primary_pairs", "primary_tests", "shadow_rays", "shadow_pairs", "shadow_tests", "loop_vs_render_mismatch")


def make(name):
    """Both builds run the same command (render() for the PPM, the replicated loop for records and
    Statistics); the reference-flag build's artefacts go under the "ref"/"ref_*" keys and into
    <cfg>.ref.records.npz (a seeded sample, or every pixel for small configs)."""
    cfg = configs.CONFIGS[name]
    os.makedirs(SCRATCH, exist_ok=True)
    W, H = cfg["W"], cfg["H"]
    small = W * H <= SMALL
    out = {}
    for build, binary in (("ref", REF), ("exact", REF_EXACT)):
        p_ppm = os.path.join(SCRATCH, "%s.%s.ppm" % (name, build))
        p_rec = os.path.join(SCRATCH, "%s.%s.records.bin" % (name, build))
        p_dump = os.path.join(SCRATCH, "%s.%s" % (name, build))
        j = run(binary, cfg, ["--out", p_ppm, "--stats", "--records", p_rec, "--dump", p_dump])
        rec = np.fromfile(p_rec, dtype=REC_DTYPE)
        assert rec.size == W * H
        out[build] = dict(j=j, ppm=open(p_ppm, "rb").read(), rec=rec, scene=_scene_hashes(p_dump))
        for suf in (".tri48", ".norm36", ".nodes32", ".prim64"):
            os.remove(p_dump + suf)
        os.remove(p_ppm)
        os.remove(p_rec)
    j_ref, j_ex = out["ref"]["j"], out["exact"]["j"]
    ppm_ref, ppm_ex = out["ref"]["ppm"], out["exact"]["ppm"]
    a_ref = np.frombuffer(ppm_ref, dtype=np.uint8)
    a_ex = np.frombuffer(ppm_ex, dtype=np.uint8)
    diff = (a_ref.astype(np.int16) - a_ex.astype(np.int16))
    meta = {
        "config": name,
        "cfg": cfg,
        "generator": "oracle/_ref/ref_render{,_exact} via tests/golden/make_golden.py",
        "n_tri": j_ex["n_tri"], "n_nodes": j_ex["n_nodes"],
        "exact": {k: j_ex[k] for k in ("rays", "hits") + STAT_KEYS},
        "ref": {k: j_ref[k] for k in ("rays", "hits") + STAT_KEYS},
        "basis": {"dir": j_ex["basis_dir"], "u": j_ex["basis_u"], "v": j_ex["basis_v"]},
        "pose": {"eye": j_ex["eye"], "sun": j_ex["sun"]},
        "ref_basis": {"dir": j_ref["basis_dir"], "u": j_ref["basis_u"], "v": j_ref["basis_v"]},
        "ref_pose": {"eye": j_ref["eye"], "sun": j_ref["sun"]},
        "ref_n_nodes": j_ref["n_nodes"],
        "ref_scene": out["ref"]["scene"],
        "ppm_sha256": {"exact": sha(ppm_ex), "ref": sha(ppm_ref)},
        "ppm_bytes_differing_ref_vs_exact": int(np.count_nonzero(diff)),
        "ppm_max_abs_diff_ref_vs_exact": int(np.abs(diff).max()) if diff.size else 0,
        "ref_render_ms_8threads": j_ref["render_ms_median"],
    }
    meta.update(out["exact"]["scene"])
    rec = out["exact"]["rec"]
    keep = _sample(rec, small)
    _save_records(os.path.join(HERE, name + ".records.npz"), rec, keep, W)
    meta["records"] = {"count": int(keep.size), "sampled": not small, "seed": SEED}
    rec_r = out["ref"]["rec"]
    keep_r = _sample(rec_r, small)
    _save_records(os.path.join(HERE, name + ".ref.records.npz"), rec_r, keep_r, W)
    meta["ref_records"] = {"count": int(keep_r.size), "sampled": not small, "seed": SEED}
    if small:
        with open(os.path.join(HERE, name + ".exact.ppm.gz"), "wb") as f:
            f.write(gzip.compress(ppm_ex, mtime=0))
        ref_gz = os.path.join(HERE, name + ".ref.ppm.gz")
        if ppm_ref != ppm_ex:
            with open(ref_gz, "wb") as f:
                f.write(gzip.compress(ppm_ref, mtime=0))
        elif os.path.exists(ref_gz):
            os.remove(ref_gz)
    with open(os.path.join(HERE, name + ".json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
        f.write("\n")
    print(name, meta["exact"]["rays"], meta["exact"]["hits"], meta["ppm_bytes_differing_ref_vs_exact"], flush=True)


ORBIT_VIEWS = 128          # bench.step_views: frame f of an F-frame step is ONE rotation by f x 360 / F degrees;
                          # F = 16N frames at N = 1, 2, 4, 8 GPUs are all among k x 360 / 128, k = 0..127


def orbit_step_deg(f, F):
    """Float32 step (degrees) of frame f of an F-frame bench step -- the same expression as
    bench.step_views (an exactly rounded double, then float32)."""
    return np.float32(f * 360.0 / F)


def make_orbit(name, views=ORBIT_VIEWS):
    """Reference PPM sha256, rays/hits (render.hpp:155) and traversal Statistics
    (single_ray_traverser.hpp:132-135) of every orbit view bench.py can time for config `name`
    (anim.cpp:76-110: the camera and sun rotated about z by the reference's own Transform,
    transform.hpp:67-112), from BOTH reference builds: the contraction-free one at the top level
    of each entry and the reference-flag one under "ref".  Only hashes and counts are stored:
    tests/golden/orbit/<name>.json, keyed by the float32 step's hex bits.  The statistics give the
    algorithmic bytes of every frame bench.py times (bench.roofline_step)."""
    cfg = configs.CONFIGS[name]
    (ax, ay, az), _ = configs.BENCH_ORBIT
    os.makedirs(SCRATCH, exist_ok=True)
    os.makedirs(os.path.join(HERE, "orbit"), exist_ok=True)
    steps = [orbit_step_deg(k, views) for k in range(views)]
    entries = {}
    for build, binary in (("exact", REF_EXACT), ("ref", REF)):
        out = os.path.join(SCRATCH, name + ".orbit")
        cmd = ([binary] + configs.cli_args(cfg) + ["--orbit", repr(ax), repr(ay), repr(az), "0", "0",
               "--orbit-views", ",".join(repr(float(s)) for s in steps), "--out", out, "--stats"])
        lines = subprocess.run(cmd, check=True, capture_output=True, text=True).stdout.strip().splitlines()
        assert len(lines) == views, (name, len(lines))
        for k, (s, line) in enumerate(zip(steps, lines)):
            j = json.loads(line)
            ppm = out + ".%d.ppm" % k
            key = "%08x" % int(np.asarray(s, np.float32).view(np.uint32))
            e = {"sha256": sha(ppm), "rays": j["rays"], "hits": j["hits"], "eye": j["eye"], "sun": j["sun"],
                 "stats": {k2: j[k2] for k2 in STAT_KEYS}}
            if build == "exact":
                e.update({"k": k, "step_deg": float(s)})
                entries[key] = e
            else:
                entries[key]["ref"] = e
            os.remove(ppm)
        print(name, build, "orbit views", views, flush=True)
    meta = {"config": name, "axis": [ax, ay, az], "views": views,
            "generator": "oracle/_ref/ref_render{_exact,} --orbit-views --stats via tests/golden/make_golden.py --orbit",
            "rule": "view k = the config camera + sun rotated once by float32(k * 360 / views) degrees about "
                    "axis (Transform::rotate, transform.hpp:67-112; anim.cpp:76-88); PPM as static.cpp:135-147; "
                    "top level = contraction-free build, 'ref' = reference CMake flags",
            "by_step_bits": entries}
    with open(os.path.join(HERE, "orbit", name + ".json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
        f.write("\n")


if __name__ == "__main__":
    if sys.argv[1:2] == ["--orbit"]:
        for n in sys.argv[2:]:
            make_orbit(n)
        sys.exit(0)
    names = sys.argv[1:] or list(configs.CONFIGS)
    for n in names:
        make(n)
