"""A/B probe: per-top-level-object lane/wave test counts of world_cast (libjsrt_dbg.so, -DJSRT_DBG_COUNT).

    JSRT_LIB=.../libjsrt_dbg.so python tools/probe/dbg_counts.py [scene] [W H spp depth]
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
for name, base in (("extend", 0), ("shadow", 128)):
    rays, waves = buf[base + 126], buf[base + 127]
    print(f"{name}: rays {rays} waves {waves} ({rays / max(waves, 1):.1f} lanes/wave)")
    tl = tw = 0
    for i in range(63):
        l, w = buf[base + 2 * i], buf[base + 2 * i + 1]
        if w:
            tl += l
            tw += w
            print(f"  obj {i:2d}: lanes/ray {l / rays:.3f}  waves/wave {w / waves:.3f}  lane-util {l / (w * 64):.3f}")
    print(f"  total: object tests/ray {tl / rays:.2f}, object passes/wave {tw / waves:.2f}")
print("stage_ms", {k: round(v, 2) for k, v in st["stage_ms"].items()})
