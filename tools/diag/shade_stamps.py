"""(timing experiment) Per-phase cycles of k_shade (analytic chain profile) from a library built with
-DJSRT_X_STAMPS (python -m jsraytracer_amd.build --variant xst --profiles 0 -DJSRT_X_STAMPS):
phases 0 ray loads, 1 shade_node, 2 block_append2 (barriers + atomic), 3 fix record + stores (to retired).
    JSRT_LIB=.../libjsrt_xst.so python tools/diag/shade_stamps.py"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    import jsraytracer_amd as jr
    from oracle import pyoracle
    L = jr._native.lib()
    L.jsrt_x_stamps.argtypes = [ctypes.c_void_p]
    sc = jr.Scene(pyoracle.golden_scene("cornell_box_path"), device=0)
    buf = (ctypes.c_ulonglong * 16)()
    tile = torch.zeros(1024 * 1024, dtype=torch.int32, device="cuda:0")
    for rep in range(3):
        st = sc.render_device(tile.data_ptr(), width=1024, height=1024, spp=64, max_depth=8, kind=1, seed=1,
                              stage_events=jr._native.EVENTS_ONE_STREAM)
        L.jsrt_x_stamps(buf)
        v = list(buf)
        names = ["ray loads", "shade_node", "block_append2", "stores (retired)"]
        print(f"frame {rep}: k_shade {st['stage_ms']['k_shade']:.2f} ms; per sampled wave (cycles):",
              {names[k]: round(v[k] / max(v[8 + k], 1)) for k in range(4)},
              "waves", [v[8 + k] for k in range(4)], flush=True)


if __name__ == "__main__":
    main()
