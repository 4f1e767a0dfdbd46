import os, sys, numpy as np, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import voxelraytracer_amd as vrt
import oracle
n, w, h = 128, 256, 144
pos = (-29.11317847012795, 56.38993520074992, -26.065439917928515)
rot = (31.46615520302214, 67.1665486975383, 0.0)
rng = np.random.default_rng(sum(map(ord, "refraction")) + n)
for k in range(77):
    p_ = tuple(float(x) for x in rng.uniform(-0.5 * n, 0.5 * n, 3)); r_ = (float(rng.uniform(-80, 80)), float(rng.uniform(-180, 180)), 0.0)
    st = float(rng.uniform(0.0, 50.0))
assert p_ == pos and r_ == rot, (p_, r_)
vox = vrt.build_scene("refraction", n)
cam = vrt.make_camera(w, h, pos=pos, rot=rot)
p = vrt.default_params(4, 4, time=77.0, sun_dir=vrt.sun_dir(st))
r = vrt.Renderer(0); r.set_certified(1); r.upload_volume(vox, n)
exact, hits, _ = r.render(cam, p)
out = torch.empty((h, w, 4), dtype=torch.float32, device="cuda")
r.render_rows_async(cam, p, 0, h, 1, out.data_ptr(), 0, 0); torch.cuda.synchronize()
fast = out.cpu().numpy()
y, x = 134, 129
print("exact", exact[y, x], "fast", fast[y, x])
print("hit", hits[y, x])
ro, ho, _ = oracle.render(cam, vox, n, p, row0=y, rows=1, row_step=1)
print("oracle", ro[0, x], ho[0, x] if ho is not None else None)
# neighbours
for dx in (-1, 0, 1):
    print(dx, exact[y, x+dx], fast[y, x+dx])
