"""Writes cuda-raytrace_amd/scenes/killeroo-proxy.pbrt and its mesh include
(scenes/geometry/figure.pbrt) from pmrender.scenes.figure_mesh, so the .pbrt
file and the in-code figure_scene() describe the same triangles bit for bit.

usage: python tools/make_killeroo_proxy.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-raytrace_amd"))
from pmrender import scenes  # noqa: E402

SCENES = os.path.join(ROOT, "cuda-raytrace_amd", "scenes")


def main():
    P, idx = scenes.figure_mesh()
    os.makedirs(os.path.join(SCENES, "geometry"), exist_ok=True)
    with open(os.path.join(SCENES, "geometry", "figure.pbrt"), "w") as f:
        f.write("# Procedural killeroo substitute (pmrender/scenes.py figure_mesh, written by\n"
                "# tools/make_killeroo_proxy.py): %d triangles, coordinates multiples of 1/64.\n" % len(idx))
        f.write('Shape "trianglemesh" "integer indices" [\n')
        for i in range(0, len(idx), 8):
            f.write("  " + " ".join("%d %d %d" % tuple(t) for t in idx[i:i + 8]) + "\n")
        f.write(']\n  "point P" [\n')
        for i in range(0, len(P), 4):
            f.write("  " + "   ".join(" ".join(repr(float(c)) for c in p) for p in P[i:i + 4]) + "\n")
        f.write("]\n")
    lines = [
        "# Killeroo substitute (pbrt-v2's killeroo scenes and mesh are not in the",
        "# container): the Cornell enclosure and ceiling light with two instances of a",
        "# procedural closed mesh (geometry/figure.pbrt) through ObjectBegin /",
        "# ObjectInstance, i.e. CreateCudaShape + CudaObjectInstance. Same scene as",
        "# pmrender/scenes.py figure_scene().",
        "Scale -1 1 1",
        "LookAt 278 273 -800   278 273 0   0 1 0",
        'Camera "perspective" "float fov" [39.3]',
        'Film "image" "integer xresolution" [256] "integer yresolution" [256] "string filename" "killeroo-proxy.pfm"',
        'Renderer "cuda" "string rendername" "photonmapping" "integer paths" [262144] "integer passes" [1]',
        "",
        "WorldBegin",
        'Include "cornell-walls.pbrt"',
        'Include "cornell-light.pbrt"',
        'ObjectBegin "figure"',
        '  Material "matte" "rgb Kd" [0.5 0.5 0.8]',
        '  Include "geometry/figure.pbrt"',
        "ObjectEnd",
    ]
    for t in scenes.FIGURE_INSTANCES:
        lines += ["AttributeBegin", "  Translate %g %g %g" % t, '  ObjectInstance "figure"', "AttributeEnd"]
    lines.append("WorldEnd")
    with open(os.path.join(SCENES, "killeroo-proxy.pbrt"), "w") as f:
        f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
