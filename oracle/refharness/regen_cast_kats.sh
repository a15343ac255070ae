#!/bin/sh
# TEST INFRASTRUCTURE: regenerate tests/golden/casts/ (World.cast known answers) from the reference
# itself (needs /root/reference + node), for every golden scene.
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
OUT=$(cd "$HERE/../.." && pwd)/tests/golden/casts
SCENES=$(ls "$HERE/../../tests/golden/scenes" | sed 's/\.jsrt\.gz$//')
rm -rf "$OUT"
node "$HERE/make_cast_kats.js" "$OUT" $SCENES
gzip -9 -n -f "$OUT"/*.json
