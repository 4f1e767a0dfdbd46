#!/usr/bin/env python3
"""Generate tests/golden/atlas/atlas_ref128.npz — the reference's own material textures as data.

The reference builds its material atlas from four PNG tiles (src/main.cpp:187-193:
`Atlas(256, 128)` + AddTexture stone128, dirt128, glass128, grass128 from res/textures/). This
script decodes those files (PIL, RGBA) and lays them out as the ABI's atlas (vrt.h "textured
mode": 256x256 RGBA8, row 0 = bottom, material slot (texX, texY) of voxel.glsl:64-67 at columns
[texX*128, ...), rows [256-(texY+1)*128, ...)), exactly as voxelraytracer_amd.load_atlas does.
Only the decoded pixels are committed (data, not source); the SHA-256 of every PNG read is kept
beside them as provenance. The slot placement is Greet's Atlas (un-vendored): build-defined, see
DESIGN.md §4 "Textured mode".
Usage (needs /root/reference, i.e. this container, not the GPU box):
    python tests/golden/make_atlas_ref.py [texture_dir]
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import voxelraytracer_amd as vrt  # noqa: E402

OUT = os.path.join(HERE, "atlas", "atlas_ref128.npz")


def main():
    tex_dir = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/res/textures"
    atlas = vrt.load_atlas(tex_dir, "128", 256)
    sha = {}
    for name in vrt.ATLAS_SLOTS:
        with open(os.path.join(tex_dir, f"{name}128.png"), "rb") as f:
            sha[f"{name}128.png"] = hashlib.sha256(f.read()).hexdigest()
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    meta = dict(atlas_size=256, atlas_texture_size=128, slots=vrt.ATLAS_SLOTS, png_sha256=sha,
                source="res/textures/{stone,dirt,glass,grass}128.png via main.cpp:187-193")
    np.savez_compressed(OUT, atlas=atlas, meta=np.array(json.dumps(meta)))
    rs, cs = vrt.atlas_slot_rows(256, 128, *vrt.ATLAS_SLOTS["glass"])
    print(OUT, "glass alpha values:", np.unique(atlas[rs, cs, 3]))


if __name__ == "__main__":
    main()
