#!/bin/sh
# TEST INFRASTRUCTURE: regenerate tests/golden/ from the reference itself (needs /root/reference + node).
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
OUT=$(cd "$HERE/../.." && pwd)/tests/golden
rm -rf "$OUT/scenes" "$OUT/images" "$OUT/index.json"
node "$HERE/make_goldens.js" "$HERE/spec_golden.json" "$OUT"
node "$HERE/make_kats.js" > "$OUT/kats.json"
gzip -9 -n -f "$OUT"/scenes/*.jsrt
