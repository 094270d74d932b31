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


def make(name):
    cfg = configs.CONFIGS[name]
    os.makedirs(SCRATCH, exist_ok=True)
    W, H = cfg["W"], cfg["H"]
    small = W * H <= SMALL
    big = cfg["proc"] > 1000
    p_ref = os.path.join(SCRATCH, name + ".ref.ppm")
    p_ex = os.path.join(SCRATCH, name + ".exact.ppm")
    p_rec = os.path.join(SCRATCH, name + ".records.bin")
    p_dump = os.path.join(SCRATCH, name)
    j_ref = run(REF, cfg, ["--out", p_ref] + ([] if big else ["--stats"]))
    extra = ["--out", p_ex, "--stats", "--records", p_rec]
    if not big:
        extra += ["--dump", p_dump]
    j_ex = run(REF_EXACT, cfg, extra)

    ppm_ref = open(p_ref, "rb").read()
    ppm_ex = open(p_ex, "rb").read()
    a_ref = np.frombuffer(ppm_ref, dtype=np.uint8)
    a_ex = np.frombuffer(ppm_ex, dtype=np.uint8)
    diff = (a_ref.astype(np.int16) - a_ex.astype(np.int16))
    meta = {
        "config": name,
        "cfg": cfg,
        "generator": "oracle/_ref/ref_render{,_exact} via tests/golden/make_golden.py",
        "n_tri": j_ex["n_tri"], "n_nodes": j_ex["n_nodes"],
        "exact": {k: j_ex[k] for k in ("rays", "hits", "primary_pairs", "primary_tests", "shadow_rays",
                                       "shadow_pairs", "shadow_tests", "loop_vs_render_mismatch")},
        "ref": {k: j_ref[k] for k in ("rays", "hits")},
        "basis": {"dir": j_ex["basis_dir"], "u": j_ex["basis_u"], "v": j_ex["basis_v"]},
        "pose": {"eye": j_ex["eye"], "sun": j_ex["sun"]},
        "ppm_sha256": {"exact": sha(ppm_ex), "ref": sha(ppm_ref)},
        "ppm_bytes_differing_ref_vs_exact": int(np.count_nonzero(diff)),
        "ppm_max_abs_diff_ref_vs_exact": int(np.abs(diff).max()) if diff.size else 0,
        "ref_render_ms_8threads": j_ref["render_ms_median"],
    }
    if "primary_pairs" in j_ref:
        meta["ref"].update({k: j_ref[k] for k in ("primary_pairs", "primary_tests", "shadow_pairs", "shadow_tests")})
    if not big:
        meta["tri48_sha256"] = sha(p_dump + ".tri48")
        meta["norm36_sha256"] = sha(p_dump + ".norm36")
        meta["bvh_canonical_sha256"] = canonical_bvh_sha(open(p_dump + ".nodes32", "rb").read(),
                                                         open(p_dump + ".prim64", "rb").read())
    # records (contraction-free reference)
    rec = np.fromfile(p_rec, dtype=REC_DTYPE)
    assert rec.size == W * H
    if small:
        keep = np.arange(rec.size)
    else:
        rng = np.random.default_rng(SEED)
        hit = np.flatnonzero(rec["prim"] >= 0)
        other = np.flatnonzero(rec["prim"] < 0)
        keep = np.sort(np.concatenate([rng.choice(hit, min(SAMPLE_HITS, hit.size), replace=False),
                                       rng.choice(other, min(SAMPLE_OTHER, other.size), replace=False)]))
    r = rec[keep]
    np.savez_compressed(os.path.join(HERE, name + ".records.npz"),
                        pixel=(r["j"].astype(np.uint64) * W + r["i"]).astype(np.uint32),
                        prim=r["prim"], t=r["t"], u=r["u"], v=r["v"], shadow=r["shadow"],
                        rgb=np.stack([r["r"], r["g"], r["b"]], axis=1))
    meta["records"] = {"count": int(keep.size), "sampled": not small, "seed": SEED}
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
    for p in (p_ref, p_ex, p_rec):
        os.remove(p)
    print(name, meta["exact"]["rays"], meta["exact"]["hits"], meta["ppm_bytes_differing_ref_vs_exact"], flush=True)


def add_scene_hashes(name):
    """Scene checksums for a config whose fixture was made without them (the 10M-triangle C5):
    the reference's rotated triangles, normals and canonical BVH, dumped by the contraction-free
    reference harness at a 1x1 frame (the dump does not depend on the frame size) and hashed
    with the oracle's C serialiser (same byte stream as canonical_bvh_sha)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    cfg = configs.CONFIGS[name]
    os.makedirs(SCRATCH, exist_ok=True)
    p_dump = os.path.join(SCRATCH, name)
    run(REF_EXACT, cfg, ["--size", "1", "1", "--out", os.devnull, "--dump", p_dump])
    nodes = np.fromfile(p_dump + ".nodes32", dtype=np.uint32)
    prim = np.fromfile(p_dump + ".prim64", dtype=np.uint64)
    path = os.path.join(HERE, name + ".json")
    meta = json.load(open(path))
    meta["tri48_sha256"] = sha(p_dump + ".tri48")
    meta["norm36_sha256"] = sha(p_dump + ".norm36")
    meta["bvh_canonical_sha256"] = oracle.canonical_bvh_sha(nodes, prim)
    with open(path, "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
        f.write("\n")
    for suf in (".tri48", ".norm36", ".nodes32", ".prim64"):
        os.remove(p_dump + suf)
    print(name, "scene hashes added", flush=True)


ORBIT_VIEWS = 128          # bench.step_views: frame f of an F-frame step is ONE rotation by f x 360 / F degrees;
                          # F = 16N frames at N = 1, 2, 4, 8 GPUs are all among k x 360 / 128, k = 0..127


def orbit_step_deg(f, F):
    """Float32 step (degrees) of frame f of an F-frame bench step -- the same expression as
    bench.step_views (an exactly rounded double, then float32)."""
    return np.float32(f * 360.0 / F)


def make_orbit(name, views=ORBIT_VIEWS):
    """Reference PPM sha256 + rays/hits (render.hpp:155) of every orbit view bench.py can time
    for config `name` (anim.cpp:76-110: the camera and sun rotated about z by the reference's own
    Transform, transform.hpp:67-112), from the contraction-free reference build.  Only hashes and
    counts are stored: tests/golden/orbit/<name>.json, keyed by the float32 step's hex bits."""
    cfg = configs.CONFIGS[name]
    (ax, ay, az), _ = configs.BENCH_ORBIT
    os.makedirs(SCRATCH, exist_ok=True)
    os.makedirs(os.path.join(HERE, "orbit"), exist_ok=True)
    steps = [orbit_step_deg(k, views) for k in range(views)]
    out = os.path.join(SCRATCH, name + ".orbit")
    cmd = ([REF_EXACT] + configs.cli_args(cfg) + ["--orbit", repr(ax), repr(ay), repr(az), "0", "0",
           "--orbit-views", ",".join(repr(float(s)) for s in steps), "--out", out])
    lines = subprocess.run(cmd, check=True, capture_output=True, text=True).stdout.strip().splitlines()
    assert len(lines) == views, (name, len(lines))
    entries = {}
    for k, (s, line) in enumerate(zip(steps, lines)):
        j = json.loads(line)
        ppm = out + ".%d.ppm" % k
        key = "%08x" % int(np.asarray(s, np.float32).view(np.uint32))
        entries[key] = {"k": k, "step_deg": float(s), "sha256": sha(ppm), "rays": j["rays"], "hits": j["hits"],
                        "eye": j["eye"], "sun": j["sun"]}
        os.remove(ppm)
    meta = {"config": name, "axis": [ax, ay, az], "views": views,
            "generator": "oracle/_ref/ref_render_exact --orbit-views via tests/golden/make_golden.py --orbit",
            "rule": "view k = the config camera + sun rotated once by float32(k * 360 / views) degrees about "
                    "axis (Transform::rotate, transform.hpp:67-112; anim.cpp:76-88); PPM as static.cpp:135-147",
            "by_step_bits": entries}
    with open(os.path.join(HERE, "orbit", name + ".json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
        f.write("\n")
    print(name, "orbit views", views, flush=True)


if __name__ == "__main__":
    if sys.argv[1:2] == ["--orbit"]:
        for n in sys.argv[2:]:
            make_orbit(n)
        sys.exit(0)
    if sys.argv[1:2] == ["--scene-hashes"]:
        for n in sys.argv[2:]:
            add_scene_hashes(n)
        sys.exit(0)
    names = sys.argv[1:] or list(configs.CONFIGS)
    for n in names:
        make(n)
