#!/usr/bin/env python3
"""Writes scenes/CBlucy_standin.dae, the stand-in for the north-star scene dae/sky/CBlucy.dae
(absent from the reference checkout, SURVEY.md §8d "CBlucy stand-in"): the Cornell box, light and
camera of scenes/CBbunny.dae with the bunny mesh subdivided once 1 -> 4 at edge midpoints
(28,576 -> 114,304 triangles, 14,290 -> 57,154 vertices), written as a VERTEX-only polylist with
positions printed %.7g. Deterministic: same input, same bytes.

usage: gen_standin.py [in.dae] [out.dae]
"""
import os
import sys
import xml.etree.ElementTree as ET

NS = "http://www.collada.org/2005/11/COLLADASchema"
Q = "{%s}" % NS


def subdivide(pos, tris):
    """pos: list of (x, y, z) floats; tris: list of (a, b, c). New vertex per edge in order of
    first use (faces in order, edges ab, bc, ca); faces (a,ab,ca) (ab,b,bc) (ca,bc,c) (ab,bc,ca)."""
    pos = list(pos)
    mid = {}

    def m(a, b):
        k = (a, b) if a < b else (b, a)
        if k not in mid:
            pa, pb = pos[a], pos[b]
            pos.append(tuple((pa[i] + pb[i]) / 2 for i in range(3)))
            mid[k] = len(pos) - 1
        return mid[k]

    out = []
    for a, b, c in tris:
        ab, bc, ca = m(a, b), m(b, c), m(c, a)
        out += [(a, ab, ca), (ab, b, bc), (ca, bc, c), (ab, bc, ca)]
    return pos, out


def main():
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(here, "scenes", "CBbunny.dae")
    dst = sys.argv[2] if len(sys.argv) > 2 else os.path.join(here, "scenes", "CBlucy_standin.dae")
    ET.register_namespace("", NS)
    tree = ET.parse(src)
    root = tree.getroot()
    geom = None
    for g in root.iter(Q + "geometry"):
        pl = g.find(f"{Q}mesh/{Q}polylist")
        if pl is not None and int(pl.get("count")) > 1000:
            geom = g
    if geom is None:
        raise SystemExit("no large mesh in " + src)
    mesh = geom.find(Q + "mesh")
    pl = mesh.find(Q + "polylist")
    verts_el = mesh.find(Q + "vertices")
    pos_src_id = verts_el.find(Q + "input").get("source")[1:]
    pos_src = [s for s in mesh.findall(Q + "source") if s.get("id") == pos_src_id][0]
    fa = pos_src.find(Q + "float_array")
    vals = [float(t) for t in fa.text.split()]
    pos = [tuple(vals[i:i + 3]) for i in range(0, len(vals), 3)]
    inputs = pl.findall(Q + "input")
    stride = len(inputs)
    voff = [int(i.get("offset")) for i in inputs if i.get("semantic") == "VERTEX"][0]
    vcount = [int(t) for t in pl.find(Q + "vcount").text.split()]
    if any(v != 3 for v in vcount):
        raise SystemExit("non-triangle polygon")
    idx = [int(t) for t in pl.find(Q + "p").text.split()]
    tris = [tuple(idx[(3 * f + k) * stride + voff] for k in range(3)) for f in range(len(vcount))]
    pos2, tris2 = subdivide(pos, tris)
    fa.text = " ".join("%.7g" % c for p in pos2 for c in p)
    fa.set("count", str(3 * len(pos2)))
    acc = pos_src.find(f"{Q}technique_common/{Q}accessor")
    if acc is not None:
        acc.set("count", str(len(pos2)))
    for s in list(mesh.findall(Q + "source")):      # VERTEX-only: drop normals / uvs
        if s.get("id") != pos_src_id:
            mesh.remove(s)
    for i in inputs:
        if i.get("semantic") != "VERTEX":
            pl.remove(i)
        else:
            i.set("offset", "0")
    pl.set("count", str(len(tris2)))
    pl.find(Q + "vcount").text = " ".join("3" for _ in tris2)
    pl.find(Q + "p").text = " ".join(str(v) for t in tris2 for v in t)
    tree.write(dst, encoding="utf-8", xml_declaration=True)
    print(f"{dst}: {len(pos2)} vertices, {len(tris2)} triangles (from {len(pos)} / {len(tris)})")


if __name__ == "__main__":
    main()
