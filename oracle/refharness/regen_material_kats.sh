#!/bin/sh
# TEST INFRASTRUCTURE: regenerate tests/golden/material/ (material_data and SDF.distance known answers)
# from the reference itself (needs /root/reference + node), for every golden scene, over the rays of
# tests/golden/casts/.
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(cd "$HERE/../.." && pwd)
OUT=$ROOT/tests/golden/material
SCENES=$(ls "$ROOT/tests/golden/scenes" | sed 's/\.jsrt\.gz$//')
rm -rf "$OUT"
node "$HERE/make_material_kats.js" "$ROOT/tests/golden/casts" "$OUT" $SCENES
gzip -9 -n -f "$OUT"/*.json
