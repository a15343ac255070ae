"""(diagnostic) Small renders of a few golden scenes against the oracle, with stats: a fast check of a build."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch  # noqa: F401
    import jsraytracer_amd as jr
    from oracle import pyoracle
    for name, W, H, spp in (("ASimpleScene", 32, 32, 2), ("cornell_box_path", 48, 40, 3), ("heart", 32, 32, 2),
                            ("bunny", 32, 24, 1)):
        blob = pyoracle.golden_scene(name)
        depth = pyoracle.scene_header(blob)["max_depth"]
        rgba, col, st = jr.Scene(blob, device=0).render(W, H, spp, depth, 1, 3)
        ocol, orgba, _ = pyoracle.render(blob, W, H, spp, depth, 1, 3)
        bad = (rgba != orgba).any(-1)
        print(name, "differing", int(bad.sum()), "of", bad.size, "attempts", st["attempts"], "launches",
              st["stage_launches"], {k: round(v, 3) for k, v in st["stage_ms"].items() if v}, flush=True)


if __name__ == "__main__":
    main()
