#!/bin/sh
# TEST INFRASTRUCTURE: regenerate tests/golden/meshes/ from the reference itself (needs /root/reference + node).
#   OBJ and MTL sources (the reference's own asset files, gzipped), the template skeleton blobs, the
#   topology digests of the reference-built BVHs (one per BVHAggregate.build), and reference renders of
#   every mesh scene (full blobs are megabytes and never committed: tests rebuild them natively from
#   skeleton + OBJ + MTL).
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
REPO=$(cd "$HERE/../.." && pwd)
OUT=$REPO/tests/golden/meshes
REF=${JSRT_REFERENCE:-/root/reference}
SCENES="bunny dragon utah_teapot tie_fighter x-wing starwars"
TMP=$(mktemp -d)
mkdir -p "$OUT/images"
node --max-old-space-size=16000 "$HERE/make_mesh_fixtures.js" "$TMP" $SCENES
node --max-old-space-size=16000 "$HERE/make_goldens.js" "$HERE/spec_mesh.json" "$TMP/gold"
for s in $SCENES; do gzip -9 -n -c "$TMP/$s.skel.jsrt" > "$OUT/$s.skel.jsrt.gz"; done
rm -f "$OUT"/images/*
cp "$TMP"/gold/images/* "$OUT/images/"
cp "$TMP/gold/index.json" "$OUT/index.json"
python3 - "$TMP" "$OUT" "$REF" $SCENES <<'PY'
import gzip, json, os, sys
tmp, out, ref, scenes = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4:]
sys.path.insert(0, os.path.join(out, "..", ".."))  # tests/
import mesh_topology as mt
topo = {}
for s in scenes:
    full = open(f"{tmp}/{s}.full.jsrt", "rb").read()
    trees = []
    for t in json.load(open(f"{tmp}/{s}.json"))["trees"]:
        sha, nodes, depth, tris = mt.digest(full, t["bvh_object_full"])
        assert (nodes, depth, tris) == (t["nodes"], t["max_depth"], t["triangles"])
        for f in [t["obj"]] + t["mtl"]:
            dst = os.path.join(out, os.path.basename(f) + ".gz")
            if not os.path.exists(dst) or gzip.open(dst).read() != open(os.path.join(ref, f), "rb").read():
                with open(os.path.join(ref, f), "rb") as src, gzip.GzipFile(dst, "wb", 9, mtime=0) as g:
                    g.write(src.read())
        trees.append(dict(obj=t["obj"], obj_fixture=os.path.basename(t["obj"]) + ".gz",
                          mtl_fixtures=[os.path.basename(m) + ".gz" for m in t["mtl"]], bvh_object=t["bvh_object"],
                          triangles=tris, nodes=nodes, max_depth=depth, sha256=sha))
    topo[s] = dict(trees[0], skeleton=f"{s}.skel.jsrt.gz", trees=trees)
json.dump(topo, open(f"{out}/topology.json", "w"), indent=1)
PY
rm -rf "$TMP"
