"""GPU debug: per-scale partial sums and argmin maps of K1 vs the CPU oracle (one golden case)."""
import ctypes
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import golden_util as gu  # noqa: E402
from oracle import photometric_oracle as O  # noqa: E402
import __graft_entry__  # noqa: E402

__graft_entry__.build()
from packnet_sfm_amd import _hip  # noqa: E402
from packnet_sfm_amd.losses import _hip_photometric as HP  # noqa: E402

case = sys.argv[1] if len(sys.argv) > 1 else "default"
z = gu.load_golden(f"loss_{case}")
kw = {k: eval(v) for k, v in zip(z["kwargs_keys"], z["kwargs_vals"])}
dev = torch.device("cuda:0")
T = lambda a: torch.from_numpy(np.ascontiguousarray(a))  # noqa: E731
nctx = sum(1 for k in z if k.startswith("ctx"))
S = kw["num_scales"]
img, K = T(z["image"]), T(z["K"])
ctxs = [T(z[f"ctx{j}"]) for j in range(nctx)]
sigs = [T(z[f"sig{i}"]) for i in range(S)]
mats = [O.pose_vec_to_mat(T(z["vec"])[:, j]) for j in range(nctx)]
B, _, H, W = img.shape

# oracle candidates (scale 0)
inv = [1.0 / (O.sigmoid_to_depth(s, kw["min_depth"], kw["max_depth"]) + 1e-8) for s in sigs]
cands = []
for j in range(nctx):
    depth = 1.0 / inv[0].clamp(min=1e-6)
    w = O.synthesize(ctxs[j], depth, K, K, mats[j])
    cands.append(O.photometric_map(w, img, kw["ssim_loss_weight"], kw["C1"], kw["C2"]))
    if kw["automask_loss"]:
        cands.append(O.photometric_map(ctxs[j], img, kw["ssim_loss_weight"], kw["C1"], kw["C2"]))
cat = torch.cat(cands, 1)
omin, oarg = cat.min(1)
print("oracle scale0 min sum", float(omin.sum()), "golden", float(z["min0"].sum()))

cfg = dict(n=S, automask=bool(kw["automask_loss"]),
           reduce_op=0 if kw["photometric_reduce_op"] == "min" else 1, ssim_w=kw["ssim_loss_weight"],
           C1=kw["C1"], C2=kw["C2"], min_depth=kw["min_depth"], max_depth=kw["max_depth"],
           clip=kw["clip_loss"], smooth_w=kw["smooth_loss_weight"])
Tm = torch.stack([m[:, :3, :] for m in mats], 0).to(dev)
kinv = HP.pinhole_inverse(K).reshape(1, 1, B, 9).expand(S, nctx, B, 9)
kref = K.reshape(1, 1, B, 9).expand(S, nctx, B, 9)
cam = torch.cat([kinv, kref, Tm.cpu().reshape(1, nctx, B, 12).expand(S, nctx, B, 12),
                 torch.zeros(S, nctx, B, 2)], -1).contiguous().to(dev)
c = HP._Call(cfg, 0, S, img.to(dev), [x.to(dev) for x in ctxs], [s.to(dev) for s in sigs], cam, None)
L = _hip.lib()
st = _hip.stream(dev)
_hip.check(L.psfm_photometric_fwd(ctypes.byref(c.params), ctypes.byref(c.inputs), ctypes.byref(c.ws), st), "fwd")
torch.cuda.synchronize()
tiles = _hip.tiles_per_image(H, W)
part = c.fbuf[: S * B * tiles].reshape(S, B * tiles).cpu()
print("hip per-scale sums", part.sum(1).tolist())
print("golden per-scale sums", [float(z[f"min{i}"].sum()) for i in range(S)])
arg = c.abuf[: S * B * H * W].reshape(S, B, H, W).cpu().long()
mism = (arg[0] != oarg).nonzero()
print("argmin mismatches scale0:", mism.shape[0], "of", B * H * W)
if mism.shape[0]:
    print(mism[:20].tolist())
    b, y, x = mism[0].tolist()
    print("oracle cands at", (b, y, x), cat[b, :, y, x].tolist(), "hip arg", int(arg[0, b, y, x]))
# per-tile comparison
ot = omin.reshape(B, H, W)
for b in range(B):
    for t in range(tiles):
        tx, ty = t % ((W + 63) // 64), t // ((W + 63) // 64)
        ref = float(ot[b, ty * 4:ty * 4 + 4, tx * 64:tx * 64 + 64].sum())
        got = float(part[0, b * tiles + t])
        if abs(ref - got) > 1e-4 * max(1.0, abs(ref)):
            print(f"tile b={b} t={t} (ty={ty},tx={tx}) oracle {ref:.6f} hip {got:.6f}")

# ---- isolate the warp: standalone HIP view_synthesis vs oracle ----
depth0 = (1.0 / inv[0].clamp(min=1e-6)).contiguous()
for j in range(nctx):
    w_ref = O.synthesize(ctxs[j], depth0, K, K, mats[j])
    out = torch.empty(B, 3, H, W, device=dev)
    camj = cam[0, j].contiguous()
    _hip.check(L.psfm_view_synthesis_fwd(B, H, W, _hip.ptr(ctxs[j].to(dev).contiguous()),
                                         _hip.ptr(depth0.to(dev)), _hip.ptr(camj), _hip.ptr(out), st), "vs")
    torch.cuda.synchronize()
    d = (out.cpu() - w_ref).abs()
    print(f"ctx{j} warp max abs err {float(d.max()):.3e} at {np.unravel_index(int(d.argmax()), d.shape)}")
