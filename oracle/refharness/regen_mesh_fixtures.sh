#!/bin/sh
# TEST INFRASTRUCTURE: regenerate tests/golden/meshes/ from the reference itself (needs /root/reference + node).
#   OBJ sources (the reference's own asset files, gzipped), the template skeleton blobs, the topology
#   digests of the reference-built BVHs, and reference renders of the dragon (whose full blob is ~47 MB
#   and is therefore never committed: tests rebuild it natively from skeleton + OBJ).
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
REPO=$(cd "$HERE/../.." && pwd)
OUT=$REPO/tests/golden/meshes
REF=${JSRT_REFERENCE:-/root/reference}
TMP=$(mktemp -d)
mkdir -p "$OUT/images"
node --max-old-space-size=16000 "$HERE/make_mesh_fixtures.js" "$TMP" bunny dragon
node --max-old-space-size=16000 "$HERE/make_goldens.js" "$HERE/spec_mesh.json" "$TMP/gold"
gzip -9 -n -c "$REF/assets/bunny2.obj" > "$OUT/bunny2.obj.gz"
gzip -9 -n -c "$REF/assets/dragon.obj" > "$OUT/dragon.obj.gz"
for s in bunny dragon; do gzip -9 -n -c "$TMP/$s.skel.jsrt" > "$OUT/$s.skel.jsrt.gz"; done
cp "$TMP"/gold/images/* "$OUT/images/"
cp "$TMP/gold/index.json" "$OUT/index.json"
python3 - "$TMP" "$OUT" <<'PY'
import json, sys
sys.path.insert(0, sys.argv[2] + "/../..")
import mesh_topology as mt
tmp, out = sys.argv[1], sys.argv[2]
topo = {}
for s in ("bunny", "dragon"):
    meta = json.load(open(f"{tmp}/{s}.json"))
    sha, nodes, depth, tris = mt.digest(open(f"{tmp}/{s}.full.jsrt", "rb").read())
    assert (nodes, depth, tris) == (meta["nodes"], meta["max_depth"], meta["triangles"])
    topo[s] = dict(meta, sha256=sha, obj_fixture=meta["obj"].split("/")[-1] + ".gz", skeleton=f"{s}.skel.jsrt.gz")
json.dump(topo, open(f"{out}/topology.json", "w"), indent=1)
PY
rm -rf "$TMP"
