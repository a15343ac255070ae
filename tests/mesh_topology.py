"""TEST INFRASTRUCTURE: read JSRT blob sections and digest a BVHAggregate's tree.

The digest walks the tree the way the reference's exporter and traversal see it (pre-order, lesser
subtree first, aggregates.js:65-87,221-222) and hashes, per node: depth, leaf flag, AABB centre and
half size (f32 bit patterns); per leaf object: the Triangle record fields the reference computes
(geometry.js:335-354: ps, v0, v1, normal, delta, d00, d11, d01, denom, area, vertex normals, UVs),
the material (its MATL record with every MaterialColor index replaced by that MCOL record's own
content key, recursively: makeMaterial's PhongMaterial from an MTL file, objloader.js:9-20) and the
shadow flag.  Two blobs with equal digests hold bit-identical trees with equal materials, so
closest-hit ties break alike and shading agrees.  Record indices (which differ between exporters) are
not hashed.
"""
import hashlib
import struct

import numpy as np

TAGS = {"OBJS": 32, "BVHN": 64, "TRIS": 256, "GEOM": 48, "CHLD": 4, "MATS": 256, "MCOL": 40, "MATL": 64}


def fourcc(s):
    return s[0] | (s[1] << 8) | (s[2] << 16) | (s[3] << 24)


def sections(blob):
    blob = bytes(blob)
    magic, version, n, _ = struct.unpack_from("<4I", blob, 0)
    assert magic == 0x5452534A and version == 1, "not a JSRT v1 blob"
    out = {}
    for i in range(n):
        tag, count, off, nbytes = struct.unpack_from("<IIQQ", blob, 16 + 24 * i)
        name = struct.pack("<I", tag).decode()
        out[name] = (count, blob[off:off + nbytes])
    return out


def objects(sec):
    cnt, raw = sec["OBJS"]
    return np.frombuffer(raw, np.int32).reshape(cnt, 8)  # kind geometry material casts first n bvh_root matrix


def bvh_objects(blob):
    o = objects(sections(blob))
    return [i for i in range(len(o)) if o[i, 0] == 3]


class _Materials:
    """Content keys of MATL / MCOL records (record indices replaced by the referenced content)."""

    def __init__(self, sec):
        self.mcol, self.matl = sec["MCOL"][1], sec["MATL"][1]
        self.kc, self.km = {}, {}

    def mc(self, i):
        if i < 0:
            return b"-"
        if i not in self.kc:
            r = self.mcol[40 * i:40 * i + 40]
            kind, a, b = struct.unpack_from("<I2i", r, 0)
            self.kc[i] = hashlib.sha256(struct.pack("<I", kind) + self.mc(a) + self.mc(b) + r[12:]).digest()
        return self.kc[i]

    def mat(self, i):
        if i < 0:
            return b"-"
        if i not in self.km:
            r = self.matl[64 * i:64 * i + 64]
            kind, *refs = struct.unpack_from("<I7i", r, 0)
            self.km[i] = hashlib.sha256(struct.pack("<I", kind) + b"".join(self.mc(x) for x in refs) + r[32:]).digest()
        return self.km[i]


def digest(blob, bvh_object=None):
    """(sha256 hex, nodes, max_depth, triangles) of a BVHAggregate's tree."""
    sec = sections(blob)
    O = objects(sec)
    if bvh_object is None:
        bvh_object = [i for i in range(len(O)) if O[i, 0] == 3][0]
    N = sec["BVHN"][1]
    C = np.frombuffer(sec["CHLD"][1], np.int32)
    G = np.frombuffer(sec["GEOM"][1], np.int32).reshape(-1, 12)
    T = sec["TRIS"][1]
    M = _Materials(sec)
    h = hashlib.sha256()
    nodes = tris = maxd = 0
    stack = [int(O[bvh_object, 6])]
    while stack:
        k = stack.pop()
        rec = N[64 * k:64 * k + 64]
        center, half = rec[0:16], rec[16:32]
        is_leaf, lesser, greater, first, n, depth = struct.unpack_from("<I5i", rec, 32)
        h.update(struct.pack("<iI", depth, is_leaf) + center + half)
        nodes += 1
        maxd = max(maxd, depth)
        if is_leaf:
            for c in C[first:first + n]:
                kind, geom, mat, casts = (int(x) for x in O[c, :4])
                assert kind == 1 and G[geom, 0] == 7, "BVH leaf object is not a Primitive over a Triangle"
                t = int(G[geom, 1])
                h.update(M.mat(mat) + struct.pack("<I", casts) + T[256 * t:256 * t + 256])
                tris += 1
        else:
            stack.append(greater)  # pre-order, lesser first
            stack.append(lesser)
    return h.hexdigest(), nodes, maxd, tris
