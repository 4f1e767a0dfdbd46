"""Diagnostic: full-size textured C3 with the reference atlas, kernel (STATS) vs oracle: list
the pixels whose hit records or colour differ."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import oracle
import voxelraytracer_amd as vrt

atlas = np.load(os.path.join(ROOT, "tests/golden/atlas/atlas_ref128.npz"))["atlas"]
vox = vrt.build_scene("refraction", 128)
cam = vrt.make_camera(1920, 1080)
p = vrt.textured_params(vrt.default_params(4, 4), atlas)
with vrt.Renderer(0) as r:
    r.upload_volume(vox, 128)
    rg, hg, sg = r.render(cam, p)
ro, ho, co = oracle.render(cam, vox, 128, p, threads=16)
bad_steps = np.argwhere(hg["steps"] != ho["steps"])
dcol = np.abs(np.clip(rg[..., :3], 0, 1) - np.clip(ro[..., :3], 0, 1)).max(-1)
bad_col = np.argwhere(dcol > 1e-4)
print("steps mismatches", len(bad_steps), "colour mismatches", len(bad_col))
print({k: (sg[k], co[k]) for k in co})
for y, x in bad_steps[:20]:
    print(y, x, "gpu", hg[y, x], rg[y, x], "oracle", ho[y, x], ro[y, x])
np.save(os.path.join(ROOT, "gpurun_out", "tex_bad.npy"), bad_steps)
