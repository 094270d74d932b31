"""Named scene/camera configurations (SURVEY.md §8(d) C1-C5 plus parity edge cases).

Every entry is the explicit input set of one render: the mesh, the `--rotate` applied by
`rotate_triangles` (render.hpp:24-44), the `Camera` (render.hpp:16-22), the sun position and
the framebuffer size.  Defaults of the single-frame app are static.cpp:39-47,72-73.

`mode` is "full" (primary + shadow + smooth shading, render.hpp:104-153) or "primary"
(primary rays only; pixel = |normalize(tri.n)|, the normal visualisation left commented
out at render.hpp:123-125 -- the C2 "primary rays only" configuration).  `robust` traverses
with the library's RobustNodeIntersector instead of render()'s FastNodeIntersector.
"""
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DATA = os.path.join(REPO, "data")
GOLDEN = os.path.join(REPO, "tests", "golden")

# static.cpp:39-47 camera + sun + rotation (dragon); README.md:11 eye/rotate for the bunny,
# with dir/up chosen so the bunny is in view.
_DRAGON = dict(obj="dragon.obj", eye=(0.0, -15.0, 2.0), dir=(0.0, 1.0, 0.0), up=(0.0, 0.0, 1.0),
               fov=60.0, sun=(-50.0, -20.0, 0.0), rotate=("x", 90.0))
_BUNNY = dict(obj="bunny.obj", eye=(0.0, 0.1, -0.3), dir=(0.0, 0.0, 1.0), up=(0.0, 1.0, 0.0),
              fov=60.0, sun=(-50.0, -20.0, 0.0), rotate=("y", -145.0))
# C5 procedural heightfield (no reference generator exists; SURVEY.md §8(d) C5 definition).
_PROC = dict(obj=None, eye=(0.5, -0.4, 0.6), dir=(0.0, 0.9, -0.55), up=(0.0, 0.0, 1.0),
             fov=60.0, sun=(-50.0, -20.0, 100.0), rotate=None)
_TINY = dict(eye=(0.2, 0.2, -3.0), dir=(0.0, 0.0, 1.0), up=(0.0, 1.0, 0.0), fov=60.0,
             sun=(-50.0, -20.0, 0.0), rotate=None)


def _cfg(base, **kw):
    d = dict(base)
    d.update(kw)
    d.setdefault("mode", "full")
    d.setdefault("proc", 0)
    d.setdefault("orbit", None)
    d.setdefault("robust", False)
    d.setdefault("tiled", False)       # a multi-GPU config defined as ONE framebuffer tiled over the GPUs
    return d


CONFIGS = {
    # C1: bunny 640x480 (CPU plumbing config of BASELINE.json configs[0])
    "bunny_640": _cfg(_BUNNY, W=640, H=480),
    # C2: bunny 1920x1080 primary rays only
    "bunny_1080_primary": _cfg(_BUNNY, W=1920, H=1080, mode="primary"),
    "bunny_1080": _cfg(_BUNNY, W=1920, H=1080),
    # C3: dragon 1920x1080 primary+shadow -- the BASELINE.json headline metric config
    "dragon_1080": _cfg(_DRAGON, W=1920, H=1080),
    "dragon_640": _cfg(_DRAGON, W=640, H=480),
    # C4: dragon 4096x4096 ("framebuffer tiled across 8x MI355X with RCCL gather": bench.py's
    # --collect auto deals its rows over the ranks)
    "dragon_4096": _cfg(_DRAGON, W=4096, H=4096, tiled=True),
    # ragged sizes (not multiples of any tile), single pixel
    "dragon_333x217": _cfg(_DRAGON, W=333, H=217),
    "bunny_97x61_primary": _cfg(_BUNNY, W=97, H=61, mode="primary"),
    "bunny_1x1": _cfg(_BUNNY, W=1, H=1),
    # procedural heightfield, small (101x101 vertices = 20,000 tris) and C5 (2237^2 = 9,999,392 tris)
    "proc_101": _cfg(_PROC, proc=101, W=320, H=240),
    # (bench_view0: bench.py's step is 16 copies of this view -- the z orbit leaves the heightfield)
    "proc_c5": _cfg(_PROC, proc=2237, W=3840, H=2160, tiled=True, bench_view0=True),
    # tiny hand-written meshes: root-is-leaf, fan triangulation / negative indices / v/vt/vn, degenerate tris
    "tri1": _cfg(_TINY, obj="@golden/tri1.obj", W=64, H=48),
    "quad": _cfg(_TINY, obj="@golden/quad.obj", W=64, H=48),
    "degenerate": _cfg(_TINY, obj="@golden/degenerate.obj", W=64, H=48),
    # leaves of 40 and 130 triangles (coincident copies: BinnedSahBuilder cannot split them,
    # binned_sah_builder.hpp:199-232) casting shadows on a floor; the shadow BVH4 stores them as
    # piece nodes (build_shadow_bvh4)
    "dupleaf": _cfg(_TINY, obj="@golden/dupleaf.obj", W=96, H=64, sun=(-30.0, -15.0, -20.0)),
    # anim.cpp:76-88 orbit poses: the C3 camera + sun after `count` Transform rotations of
    # step_deg about the axis (the bench's weak-scaling frames are this orbit about z)
    "dragon_orbit3_333x217": _cfg(_DRAGON, W=333, H=217, orbit=((0.0, 0.0, 1.0), 45.0, 3)),
    "bunny_orbit7_160x120": _cfg(_BUNNY, W=160, H=120, orbit=((0.0, 1.0, 0.0), 6.0, 7)),
    # rotate_triangles<2> (render.hpp:24-44 about z): the z axis's contraction sites --
    # the bunny turned in the image plane
    "bunny_rotz_160x120": _cfg(_BUNNY, W=160, H=120, rotate=("z", 37.0)),
    # RobustNodeIntersector traversal (node_intersectors.hpp:54-79): odd sizes
    # give exactly axis-aligned view rays (inverse +-inf), the sun on the y axis axis-aligned
    # shadow rays; reference = the harness's render loop with the library's robust intersector
    "dragon_333x217_robust": _cfg(_DRAGON, W=333, H=217, sun=(0.0, -20.0, 0.0), robust=True),
    "quad_65x49_robust": _cfg(_TINY, obj="@golden/quad.obj", W=65, H=49, robust=True),
    "degenerate_65x49_robust": _cfg(_TINY, obj="@golden/degenerate.obj", W=65, H=49, robust=True),
    "bunny_97x61_primary_robust": _cfg(_BUNNY, W=97, H=61, mode="primary", robust=True),
    "dragon_1080_robust": _cfg(_DRAGON, W=1920, H=1080, robust=True),
}

# pose(cfg, frame) / tests: the config pose rotated `frame` times by 45 degrees about z
BENCH_ORBIT = ((0.0, 0.0, 1.0), 45.0)
# bench.py: frame f of an F-frame step is the config pose rotated ONCE by orbit_step(f, F) degrees
# about BENCH_AXIS (anim.cpp:76-88's Transform) -- F views over the full turn; every view of every
# F = 16N (N = 1, 2, 4, 8) is among the 128 pinned by tests/golden/orbit/<cfg>.json
BENCH_AXIS = (0.0, 0.0, 1.0)
ORBIT_FIXTURE_VIEWS = 128


def orbit_step(f, F):
    """Float32 rotation (degrees) of frame f of an F-frame bench step: f x 360 / F, rounded once to
    double then to float32 (so equal fractions f / F give identical bits)."""
    import numpy as np
    return np.float32(f * 360.0 / F)


def obj_path(cfg):
    """Absolute path of a config's mesh (None for procedural meshes)."""
    o = cfg["obj"]
    if o is None:
        return None
    if o.startswith("@golden/"):
        return os.path.join(GOLDEN, o[len("@golden/"):])
    return os.path.join(DATA, o)


def cli_args(cfg):
    """The `./render` CLI flags (README.md:11 style) describing a config."""
    a = []
    if cfg["proc"]:
        a += ["--proc", str(cfg["proc"])]
    else:
        a += [obj_path(cfg)]
    a += ["--eye", *map(repr, cfg["eye"]), "--dir", *map(repr, cfg["dir"]), "--up", *map(repr, cfg["up"]),
          "--fov", repr(cfg["fov"]), "--sun", *map(repr, cfg["sun"]), "--size", str(cfg["W"]), str(cfg["H"])]
    if cfg["rotate"]:
        a += ["--rotate", cfg["rotate"][0], repr(cfg["rotate"][1])]
    if cfg.get("orbit"):
        (ax, ay, az), step, count = cfg["orbit"]
        a += ["--orbit", repr(ax), repr(ay), repr(az), repr(step), str(count)]
    if cfg["mode"] == "primary":
        a += ["--primary-only"]
    if cfg.get("robust"):
        a += ["--robust"]
    return a
