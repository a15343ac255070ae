"""A/B probe (libjsrt_dbg.so, -DJSRT_DBG_COUNT): per-level slot occupancy of k_shade and per-object
lane / wave test counts of world_cast.

    JSRT_LIB=.../libjsrt_dbg.so python tools/dbg_counts.py [scene] [W H spp depth]
"""
import ctypes
import sys

sys.path.insert(0, "/root/repo")
import jsraytracer_amd as jr  # noqa: E402
from jsraytracer_amd import _native  # noqa: E402
from oracle import pyoracle  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "cornell_box_path"
W, H, spp, depth = (int(x) for x in (sys.argv[2:6] if len(sys.argv) > 5 else (256, 256, 16, 8)))
sc = jr.Scene(pyoracle.golden_scene(scene), device=0)
lib = _native.lib()
buf = (ctypes.c_ulonglong * 256)()
lib.jsrt_debug_counters(buf, 256)  # reset
_, _, st = sc.render(W, H, spp, depth, 1, 1)
lib.jsrt_debug_counters(buf, 256)
n = W * H * spp
print(f"{scene} {W}x{H}x{spp} depth {depth}: per level (per path) lanes-in / hits / branches, lane fill")
for L in range(depth):
    i, h, b, w = buf[4 * L: 4 * L + 4]
    if w:
        print(f"  L{L}: in {i / n:.3f} hit {h / n:.3f} branch {b / n:.3f}  waves {w}  hit-fill {h / (64 * w):.3f}")
for name, base in (("extend", 128), ("shadow", 192)):
    rays, waves = buf[base + 62], buf[base + 63]
    print(f"{name}: rays {rays} waves {waves} ({rays / max(waves, 1):.1f} lanes/wave)")
    tl = tw = 0
    for i in range(31):
        l, w = buf[base + 2 * i], buf[base + 2 * i + 1]
        if w:
            tl += l
            tw += w
            print(f"  obj {i:2d}: lanes/ray {l / rays:.3f}  waves/wave {w / waves:.3f}  lane-util {l / (w * 64):.3f}")
    print(f"  total: object tests/ray {tl / max(rays, 1):.2f}, object passes/wave {tw / max(waves, 1):.2f}")
for name, base in (("extend", 100), ("shadow", 104)):
    ex, no, yes = buf[base], buf[base + 1], buf[base + 2]
    tot = max(ex + no + yes, 1)
    print(f"{name} f32 pre-tests: {tot} lane tests, no {no / tot:.3f} yes {yes / tot:.3f} exact {ex / tot:.4f}")
print("stage_ms", {k: round(v, 2) for k, v in st["stage_ms"].items()})
