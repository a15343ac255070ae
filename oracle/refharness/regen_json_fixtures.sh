#!/bin/sh
# TEST INFRASTRUCTURE: regenerate tests/golden/json/ from the reference itself (needs /root/reference + node):
#   <scene>.json.gz  JSON.stringify(new Serializer(test).plain()) of every golden scene (bunny_path
#                    aside: the same mesh as bunny), as tests/test_to_json.js writes tests/<scene>/test.json
#   <mesh>.obj.gz    the reference's OBJ assets those scenes load (the psdata side-channel)
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
REPO=$(cd "$HERE/../.." && pwd)
OUT=$REPO/tests/golden/json
REF=${JSRT_REFERENCE:-/root/reference}
TMP=$(mktemp -d)
SCENES=$(ls "$REPO/tests/golden/scenes" | sed 's/\.jsrt\.gz$//' | grep -v '^bunny_path$')
node --max-old-space-size=16000 "$HERE/make_json_fixtures.js" "$TMP" $SCENES
mkdir -p "$OUT"
for s in $SCENES; do gzip -9 -n -c "$TMP/$s.json" > "$OUT/$s.json.gz"; done
for o in cat heart hollow_tetrahedron star diamond; do gzip -9 -n -c "$REF/assets/$o.obj" > "$OUT/$o.obj.gz"; done
rm -rf "$TMP"
