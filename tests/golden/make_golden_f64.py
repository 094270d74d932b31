#!/usr/bin/env python3
"""Golden fixtures for the double-precision path (render<double>, anim.cpp's -d mode,
anim.cpp:146-155) from the REFERENCE's own code: oracle/_ref/ref_render_f64{,_exact} are
oracle/ref_harness.cpp compiled with Scalar = double from the unmodified headers in
/root/reference (oracle/Makefile).  Written to tests/golden/f64/:

  <cfg>.json           rays/hits, traversal statistics, camera basis / pose as 64-bit hex,
                       sha256 of the PPM (both contraction modes), of the double Triangle[]
                       (96 B each), tri_norms (72 B) and of the canonical BVH (64-B nodes)
  <cfg>.exact.ppm.gz   PPM of the contraction-free build (small configs)
  <cfg>.records.npz    per-pixel {pixel, prim, t, u, v, shadow, rgb} (float64) of the
                       contraction-free build, every pixel for small configs, else a sample
  <cfg>.ref.records.npz  the same pixels in the reference-flag build (round 5), whose scene
                       hashes, camera basis, pose and statistics are the "ref*" keys of the JSON

Command-line numbers reach the harness as decimal strings parsed with strtod, i.e. the
configs' values are double literals (as anim.cpp writes its camera).
Usage: python tests/golden/make_golden_f64.py [cfg ...]
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
sys.path.insert(0, HERE)
import configs  # noqa: E402
from make_golden import sha  # noqa: E402

OUT = os.path.join(HERE, "f64")
REF = os.path.join(REPO, "oracle", "_ref", "ref_render_f64")
REF_EXACT = os.path.join(REPO, "oracle", "_ref", "ref_render_f64_exact")
SCRATCH = os.path.join(REPO, ".scratch", "golden_f64")
SMALL = 640 * 480
SAMPLE_HITS, SAMPLE_OTHER, SEED = 4096, 1024, 12345
CONFIGS = ["bunny_640", "dragon_333x217", "dragon_1080", "dragon_4096", "bunny_97x61_primary", "degenerate", "tri1",
           "quad", "proc_101", "dragon_orbit3_333x217", "bunny_1x1"]

REC_DTYPE = np.dtype([("i", "<u4"), ("j", "<u4"), ("prim", "<i4"), ("pad0", "<u4"), ("t", "<f8"), ("u", "<f8"),
                      ("v", "<f8"), ("shadow", "<i4"), ("pad1", "<u4"), ("r", "<f8"), ("g", "<f8"), ("b", "<f8")])
assert REC_DTYPE.itemsize == 72


def canonical_bvh64_sha(nodes64: bytes, prim64: bytes) -> str:
    """sha256 of a bvh::Bvh<double> in DFS order, numbering-independent: per node 6 double
    bounds + u64 primitive_count (56 B), leaves followed by their primitive_indices (u64)."""
    raw = np.frombuffer(nodes64, dtype=np.uint8).reshape(-1, 64)
    cnt = raw[:, 48:56].copy().view(np.uint64).ravel()
    first = raw[:, 56:64].copy().view(np.uint64).ravel()
    prim = np.frombuffer(prim64, dtype=np.uint64)
    h = hashlib.sha256()
    stack = [0]
    while stack:
        k = stack.pop()
        h.update(raw[k, :56].tobytes())
        c, f = int(cnt[k]), int(first[k])
        if c:
            h.update(prim[f:f + c].tobytes())
        else:
            stack.append(f + 1)
            stack.append(f)
    return h.hexdigest()


def run(binary, cfg, extra):
    cmd = [binary] + configs.cli_args(cfg) + extra
    out = subprocess.run(cmd, check=True, capture_output=True, text=True).stdout
    return json.loads(out.strip().splitlines()[-1])


def make(name):
    cfg = configs.CONFIGS[name]
    os.makedirs(SCRATCH, exist_ok=True)
    os.makedirs(OUT, exist_ok=True)
    W, H = cfg["W"], cfg["H"]
    small = W * H <= SMALL
    p_ref = os.path.join(SCRATCH, name + ".ref.ppm")
    p_ex = os.path.join(SCRATCH, name + ".exact.ppm")
    p_rec = os.path.join(SCRATCH, name + ".records.bin")
    p_dump = os.path.join(SCRATCH, name)
    p_rrec = os.path.join(SCRATCH, name + ".ref.records.bin")
    p_rdump = os.path.join(SCRATCH, name + ".ref")
    j_ref = run(REF, cfg, ["--out", p_ref, "--stats", "--records", p_rrec, "--dump", p_rdump])
    j_ex = run(REF_EXACT, cfg, ["--out", p_ex, "--stats", "--records", p_rec, "--dump", p_dump])
    ppm_ref = open(p_ref, "rb").read()
    ppm_ex = open(p_ex, "rb").read()
    diff = np.frombuffer(ppm_ref, np.uint8).astype(np.int16) - np.frombuffer(ppm_ex, np.uint8).astype(np.int16)
    meta = {
        "config": name, "cfg": cfg, "scalar": "double",
        "generator": "oracle/_ref/ref_render_f64{,_exact} via tests/golden/make_golden_f64.py",
        "n_tri": j_ex["n_tri"], "n_nodes": j_ex["n_nodes"],
        "exact": {k: j_ex[k] for k in ("rays", "hits", "primary_pairs", "primary_tests", "shadow_rays",
                                       "shadow_pairs", "shadow_tests", "loop_vs_render_mismatch")},
        "ref": {k: j_ref[k] for k in ("rays", "hits", "primary_pairs", "primary_tests", "shadow_rays",
                                      "shadow_pairs", "shadow_tests", "loop_vs_render_mismatch")},
        "ref_basis": {"dir": j_ref["basis_dir"], "u": j_ref["basis_u"], "v": j_ref["basis_v"]},
        "ref_pose": {"eye": j_ref["eye"], "sun": j_ref["sun"]},
        "ref_scene": {"tri96_sha256": sha(p_rdump + ".tri96"), "norm72_sha256": sha(p_rdump + ".norm72"),
                      "bvh_canonical_sha256": canonical_bvh64_sha(open(p_rdump + ".nodes64", "rb").read(),
                                                                  open(p_rdump + ".prim64", "rb").read())},
        "basis": {"dir": j_ex["basis_dir"], "u": j_ex["basis_u"], "v": j_ex["basis_v"]},
        "pose": {"eye": j_ex["eye"], "sun": j_ex["sun"]},
        "ppm_sha256": {"exact": sha(ppm_ex), "ref": sha(ppm_ref)},
        "ppm_bytes_differing_ref_vs_exact": int(np.count_nonzero(diff)),
        "tri96_sha256": sha(p_dump + ".tri96"),
        "norm72_sha256": sha(p_dump + ".norm72"),
        "bvh_canonical_sha256": canonical_bvh64_sha(open(p_dump + ".nodes64", "rb").read(),
                                                    open(p_dump + ".prim64", "rb").read()),
        "ref_render_ms_8threads": j_ref["render_ms_median"],
    }
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
    np.savez_compressed(os.path.join(OUT, name + ".records.npz"),
                        pixel=(r["j"].astype(np.uint64) * W + r["i"]).astype(np.uint32),
                        prim=r["prim"], t=r["t"], u=r["u"], v=r["v"], shadow=r["shadow"],
                        rgb=np.stack([r["r"], r["g"], r["b"]], axis=1))
    meta["records"] = {"count": int(keep.size), "sampled": not small, "seed": SEED}
    rr = np.fromfile(p_rrec, dtype=REC_DTYPE)[keep]
    np.savez_compressed(os.path.join(OUT, name + ".ref.records.npz"),
                        pixel=(rr["j"].astype(np.uint64) * W + rr["i"]).astype(np.uint32),
                        prim=rr["prim"], t=rr["t"], u=rr["u"], v=rr["v"], shadow=rr["shadow"],
                        rgb=np.stack([rr["r"], rr["g"], rr["b"]], axis=1))
    if small:
        with open(os.path.join(OUT, name + ".exact.ppm.gz"), "wb") as f:
            f.write(gzip.compress(ppm_ex, mtime=0))
    with open(os.path.join(OUT, name + ".json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
        f.write("\n")
    for p in (p_ref, p_ex, p_rec, p_rrec, p_dump + ".tri96", p_dump + ".norm72", p_dump + ".nodes64", p_dump + ".prim64",
              p_rdump + ".tri96", p_rdump + ".norm72", p_rdump + ".nodes64", p_rdump + ".prim64"):
        os.remove(p)
    print(name, meta["exact"]["rays"], meta["exact"]["hits"], meta["ppm_bytes_differing_ref_vs_exact"], flush=True)


if __name__ == "__main__":
    for n in sys.argv[1:] or CONFIGS:
        make(n)
