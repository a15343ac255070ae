#!/bin/sh
# Builds the Node N-API addon (jsraytracer_amd/_build/jsrt_node.node) against libjsrt.so.
# Plain g++ against /usr/include/node (N-API 8, Node 12); no node-gyp.  libjsrt.so is found next to
# the addon through its RUNPATH ($ORIGIN).
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
OUT="$HERE/../_build"
[ -f "$OUT/libjsrt.so" ] || { echo "build libjsrt.so first (jsraytracer_amd/build.py)" >&2; exit 1; }
[ -f /usr/include/node/node_api.h ] || { echo "node headers missing: skipping the N-API addon" >&2; exit 0; }
if [ -f "$OUT/jsrt_node.node" ] && [ "$OUT/jsrt_node.node" -nt "$HERE/jsrt_node.cpp" ] && \
   [ "$OUT/jsrt_node.node" -nt "$HERE/../../include/jsrt.h" ] && [ "$OUT/jsrt_node.node" -nt "$HERE/../../include/jsrt_mesh.h" ]; then exit 0; fi
g++ -O2 -std=c++17 -fPIC -shared -Wall -Wextra -Wno-unused-parameter -Wno-missing-field-initializers \
    -DNODE_GYP_MODULE_NAME=jsrt_node -I/usr/include/node \
    "$HERE/jsrt_node.cpp" -o "$OUT/jsrt_node.node.tmp" \
    -L"$OUT" -ljsrt -Wl,-rpath,'$ORIGIN'
mv "$OUT/jsrt_node.node.tmp" "$OUT/jsrt_node.node"
