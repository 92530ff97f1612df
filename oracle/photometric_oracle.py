"""ORACLE — test infrastructure only (never imported by the product path).

CPU restatement (PyTorch-CPU, fp32, autograd) of the reference's self-supervised
photometric hot path.  Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s
`cpu_baseline` leg may import this module, and only as the checker / the CPU
baseline.  Parity of this restatement with the reference itself is pinned by the
golden fixtures in `tests/golden/` (generated from /root/reference by
`tools/gen_goldens.py`; see `tests/test_oracle_golden.py`).

Every function cites the reference line it restates (paths relative to the
reference's `packnet_sfm/`).
"""
import torch
import torch.nn.functional as F


# ---------------------------------------------------------------------------------------------------------------------
# geometry
# ---------------------------------------------------------------------------------------------------------------------
def euler_to_rot(ang):
    """R = Rx(a0) @ Ry(a1) @ Rz(a2).  geometry/pose_utils.py:8-37."""
    x, y, z = ang[:, 0], ang[:, 1], ang[:, 2]
    o, l = torch.zeros_like(z), torch.ones_like(z)
    cz, sz, cy, sy, cx, sx = z.cos(), z.sin(), y.cos(), y.sin(), x.cos(), x.sin()
    Rz = torch.stack([cz, -sz, o, sz, cz, o, o, o, l], 1).view(-1, 3, 3)
    Ry = torch.stack([cy, o, sy, o, l, o, -sy, o, cy], 1).view(-1, 3, 3)
    Rx = torch.stack([l, o, o, o, cx, -sx, o, sx, cx], 1).view(-1, 3, 3)
    return Rx.bmm(Ry).bmm(Rz)


def pose_vec_to_mat(vec):
    """[B,6] (t, euler) -> [B,4,4].  geometry/pose.py:39-46, pose_utils.py:41-51."""
    B = vec.shape[0]
    top = torch.cat([euler_to_rot(vec[:, 3:]), vec[:, :3].unsqueeze(-1)], 2)
    bottom = torch.tensor([0.0, 0.0, 0.0, 1.0], dtype=vec.dtype, device=vec.device).view(1, 1, 4).expand(B, 1, 4)
    return torch.cat([top, bottom], 1)


def scale_K(K, s):
    """geometry/camera_utils.py:16-22 (x and y scaled by the same factor, camera.py:84-108)."""
    if s == 1.0:
        return K
    K = K.clone()
    K[:, 0, 0] = K[:, 0, 0] * s
    K[:, 1, 1] = K[:, 1, 1] * s
    K[:, 0, 2] = (K[:, 0, 2] + 0.5) * s - 0.5
    K[:, 1, 2] = (K[:, 1, 2] + 0.5) * s - 0.5
    return K


def K_inverse(K):
    """Closed-form pinhole inverse.  geometry/camera.py:72-81."""
    Ki = K.clone()
    Ki[:, 0, 0] = 1.0 / K[:, 0, 0]
    Ki[:, 1, 1] = 1.0 / K[:, 1, 1]
    Ki[:, 0, 2] = -1.0 * K[:, 0, 2] / K[:, 0, 0]
    Ki[:, 1, 2] = -1.0 * K[:, 1, 2] / K[:, 1, 1]
    return Ki


def lift(depth, K):
    """Pixel grid -> camera-frame points d*K^-1[u,v,1].  camera.py:111-147, utils/image.py:218-282."""
    B, _, H, W = depth.shape
    v, u = torch.meshgrid(torch.arange(H, dtype=depth.dtype, device=depth.device),
                          torch.arange(W, dtype=depth.dtype, device=depth.device),
                          indexing="ij")
    grid = torch.stack([u, v, torch.ones_like(u)], 0).view(1, 3, -1).expand(B, 3, H * W)
    return (K_inverse(K).bmm(grid).view(B, 3, H, W)) * depth


def project_to_grid(X, K, T):
    """x = K (R X + t); normalised grid for grid_sample.  camera.py:149-190, pose.py:80-86."""
    B, _, H, W = X.shape
    Xc = T[:, :3, :3].bmm(X.view(B, 3, -1)) + T[:, :3, 3:]
    p = K.bmm(Xc)
    Z = p[:, 2].clamp(min=1e-5)
    xn = 2 * (p[:, 0] / Z) / (W - 1) - 1.0
    yn = 2 * (p[:, 1] / Z) / (H - 1) - 1.0
    return torch.stack([xn, yn], -1).view(B, H, W, 2)


FLT_EPS = 2.220446049250313e-16  # sys.float_info.epsilon, as the reference clamps with it


def fisheye_scale(cam, sw, sh):
    """Per-scale fisheye intrinsics: centre (ux, uy) scaled as (c + 0.5) s - 0.5; k, s, div kept
    (losses/multiview_photometric_loss.py:166-186 — the fork does not rescale s / div)."""
    return {"k": cam["k"], "s": cam["s"], "div": cam["div"],
            "ux": (cam["ux"] + 0.5) * sw - 0.5, "uy": (cam["uy"] + 0.5) * sh - 0.5}


def fisheye_lift(depth, cam):
    """FisheyeCamera.reconstruct(depth, frame='c') (geometry/camera.py:243-303): r_d from the
    centred, scaled pixel, theta ~= r_d (the reference's approximation), ray = tan(theta)/r_d."""
    B, _, H, W = depth.shape
    v, u = torch.meshgrid(torch.arange(H, dtype=depth.dtype, device=depth.device),
                          torch.arange(W, dtype=depth.dtype, device=depth.device), indexing="ij")
    u, v = u.reshape(1, -1), v.reshape(1, -1)
    xd = (u - cam["ux"].view(B, 1).to(depth.dtype)) / cam["s"].view(B, 1).to(depth.dtype)
    yd = (v - cam["uy"].view(B, 1).to(depth.dtype)) / cam["div"].view(B, 1).to(depth.dtype)
    rd = torch.sqrt(xd ** 2 + yd ** 2)
    r = torch.tan(rd)
    rds = torch.where(rd < FLT_EPS, torch.full_like(rd, FLT_EPS), rd)
    d = depth.view(B, -1)
    return torch.stack([(r / rds) * xd * d, (r / rds) * yd * d, d], 1).view(B, 3, H, W)


def fisheye_project_to_grid(X, cam, T):
    """c = R X + t, then FisheyeCamera.project(c, frame='c') (geometry/camera.py:305-394):
    theta = atan(r), r_d = k0 + sum_i k_i theta^i, (u, v) = (s, div) (r_d / r) (x, y) + (ux, uy),
    normalised to [-1, 1] (align_corners)."""
    B, _, H, W = X.shape
    Xc = T[:, :3, :3].bmm(X.view(B, 3, -1)) + T[:, :3, 3:]
    Z = Xc[:, 2].clamp(min=FLT_EPS)
    xn, yn = Xc[:, 0] / Z, Xc[:, 1] / Z
    r = torch.sqrt(xn ** 2 + yn ** 2)
    th = torch.atan(r)
    k = cam["k"].to(X.dtype)
    poly = k[:, 0].unsqueeze(1)
    for i in range(1, 7):
        poly = poly + k[:, i].unsqueeze(1) * torch.pow(th, i)
    rs = torch.where(r < FLT_EPS, torch.full_like(r, FLT_EPS), r)
    u = cam["s"].view(B, 1).to(X.dtype) * ((poly / rs) * xn) + cam["ux"].view(B, 1).to(X.dtype)
    v = cam["div"].view(B, 1).to(X.dtype) * ((poly / rs) * yn) + cam["uy"].view(B, 1).to(X.dtype)
    return torch.stack([2 * u / (W - 1) - 1.0, 2 * v / (H - 1) - 1.0], -1).view(B, H, W, 2)


def synthesize(ref, depth, K_tgt, K_ref, T, kink_flip_eps=0.0, grid_mask=None):
    """Inverse warp of `ref` into the target view.  geometry/camera_utils.py:27-59.  K_* are
    pinhole [B,3,3] tensors or FisheyeCamera (VADAS) intrinsics dicts.

    `kink_flip_eps` (test instrument, not the reference): sample with `bilinear_other_cell`, which
    puts every coordinate within eps of an integer into the OTHER bilinear cell — the same value,
    the other one-sided derivative: the second legitimate fp32 outcome at a kink.
    `grid_mask` (test instrument): [B,1,H,W] bool; those pixels' warp coordinates pass no gradient
    (their contribution to dL/dpose and dL/ddepth is dropped)."""
    if isinstance(K_tgt, dict):
        grid = fisheye_project_to_grid(fisheye_lift(depth, K_tgt), K_ref, T)
    else:
        grid = project_to_grid(lift(depth, K_tgt), K_ref, T)
    if grid_mask is not None:
        keep = (~grid_mask[:, 0]).unsqueeze(-1).to(grid.dtype)
        grid = grid * keep + (grid * (1 - keep)).detach()
    if kink_flip_eps > 0.0:
        return bilinear_other_cell(ref, grid, kink_flip_eps)
    return F.grid_sample(ref, grid, mode="bilinear", padding_mode="zeros", align_corners=True)


def bilinear_other_cell(ref, grid, eps):
    """grid_sample(bilinear, zeros, align_corners=True) written out, with the tap cell of every
    coordinate within `eps` of an integer n moved to the other side of n (x0 = n - 1 when the
    coordinate is >= n, x0 = n when below): continuous value, the other cell's slope."""
    B, C, H, W = ref.shape
    ix = (grid[..., 0] + 1) / 2 * (W - 1)
    iy = (grid[..., 1] + 1) / 2 * (H - 1)

    def cell(i):
        f = torch.floor(i.detach())
        r = torch.round(i.detach())
        near = (i.detach() - r).abs() < eps
        other = torch.where(i.detach() >= r, r - 1, r)
        return torch.where(near, other, f)

    x0, y0 = cell(ix), cell(iy)
    wx, wy = ix - x0, iy - y0
    flat = ref.reshape(B, C, H * W)
    out = 0.0
    for dy, wyk in ((0, 1 - wy), (1, wy)):
        for dx, wxk in ((0, 1 - wx), (1, wx)):
            xx, yy = x0 + dx, y0 + dy
            ok = (xx >= 0) & (xx <= W - 1) & (yy >= 0) & (yy <= H - 1)
            idx = (yy.clamp(0, H - 1) * W + xx.clamp(0, W - 1)).long().view(B, 1, -1).expand(B, C, -1)
            v = flat.gather(2, idx).view(B, C, *ix.shape[1:]) * ok.unsqueeze(1).to(ref.dtype)
            out = out + v * (wxk * wyk).unsqueeze(1)
    return out


# ---------------------------------------------------------------------------------------------------------------------
# photometric terms
# ---------------------------------------------------------------------------------------------------------------------
def ssim_map(x, y, C1=1e-4, C2=9e-4):
    """3x3 SSIM with reflect-1 padding.  losses/multiview_photometric_loss.py:15-54."""
    x, y = F.pad(x, (1, 1, 1, 1), mode="reflect"), F.pad(y, (1, 1, 1, 1), mode="reflect")
    box = lambda t: F.avg_pool2d(t, 3, 1)  # noqa: E731
    mx, my = box(x), box(y)
    vx = box(x * x) - mx * mx
    vy = box(y * y) - my * my
    cxy = box(x * y) - mx * my
    return ((2 * mx * my + C1) * (2 * cxy + C2)) / ((mx * mx + my * my + C1) * (vx + vy + C2))


def photometric_map(est, tgt, alpha, C1, C2):
    """alpha*mean_c clamp((1-SSIM)/2) + (1-alpha)*mean_c |est-tgt|.  multiview_photometric_loss.py:199-247."""
    l1 = (est - tgt).abs()
    if alpha <= 0.0:
        return l1
    ssim = torch.clamp((1.0 - ssim_map(est, tgt, C1, C2)) / 2.0, 0.0, 1.0)
    return alpha * ssim.mean(1, True) + (1 - alpha) * l1.mean(1, True)


def sigmoid_to_depth(s, min_depth, max_depth):
    """utils/post_process_depth.py:68-108."""
    lo = 1.0 / max(max_depth, 1e-6)
    hi = 1.0 / max(min_depth, 1e-6)
    return 1.0 / (lo + (hi - lo) * s + 1e-8)


def sigmoid_to_inv(s, min_depth, max_depth):
    """utils/post_process_depth.py:13-65 (linear branch)."""
    lo = 1.0 / max(max_depth, 1e-6)
    hi = 1.0 / max(min_depth, 1e-6)
    return lo + (hi - lo) * s


def resize_like(t, shape, mode="bilinear"):
    """utils/image.py:117-146 / 178-214 (identity when shapes agree)."""
    if tuple(t.shape[-2:]) == tuple(shape[-2:]):
        return t
    if mode == "nearest":
        return F.interpolate(t, size=tuple(shape[-2:]), mode="nearest")
    return F.interpolate(t, size=tuple(shape[-2:]), mode=mode, align_corners=True)


def smoothness(sigs, images, n):
    """Edge-aware smoothness on the sigmoid maps.  utils/depth.py:146-198, multiview_photometric_loss.py:301-327."""
    total = 0.0
    for i in range(n):
        d = sigs[i] / sigs[i].mean(2, True).mean(3, True).clamp(min=1e-6)
        I = images[i]
        wx = torch.exp(-(I[..., :-1] - I[..., 1:]).abs().mean(1, True))
        wy = torch.exp(-(I[..., :-1, :] - I[..., 1:, :]).abs().mean(1, True))
        sx = (d[..., :-1] - d[..., 1:]) * wx
        sy = (d[..., :-1, :] - d[..., 1:, :]) * wy
        total = total + (sx.abs().mean() + sy.abs().mean()) / 2 ** i
    return total / n


def num_scales(progressive_scaling, num, progress):
    """losses/loss_base.py:10-49.  The reference stores the thresholds as an np.float32 ARRAY and
    then tests them with is_list() (utils/types.py:21-23: isinstance(data, list)), which is False:
    the scale count never decreases (goldens loss_progressive_p03 / _p06 pin this)."""
    if progressive_scaling > 0.0:
        import numpy as np
        steps = np.float32([progressive_scaling * (i + 1) for i in range(num - 1)] + [1.0])
        if isinstance(steps, list):   # never true (the reference's is_list test)
            return int(num - np.searchsorted(steps, progress))
    return num


def photometric_loss(image, contexts, sigs, K, ref_K, pose_mats, mask=None, num_scales_=4,
                     ssim_loss_weight=0.85, smooth_loss_weight=0.001, C1=1e-4, C2=9e-4,
                     photometric_reduce_op="min", clip_loss=0.0, automask_loss=True,
                     min_depth=0.5, max_depth=80.0, progressive_scaling=0.0, progress=0.0, tie_flip=None,
                     kink_flip_eps=0.0, grid_mask=None):
    """MultiViewPhotometricLoss.forward restated.  losses/multiview_photometric_loss.py:331-410.

    sigs: list of [B,1,h,w] sigmoid maps (the fork feeds sigmoid outputs, :362-369);
    pose_mats: list of [B,4,4] target->context transforms.  Pinhole cameras.
    Returns (loss[1], photometric metric, smoothness, per-scale reduced maps).

    Test instruments (not the reference), for bounding the gradient at `sensitive_pixels`:
    `tie_flip`: per-scale boolean maps [B,1,h,w]; at those pixels the min-reprojection selects the
    SECOND-smallest candidate — the other legitimate fp32 outcome at a near-tie;
    `kink_flip_eps`: every warp coordinate within eps of an integer takes the other bilinear cell
    (synthesize) — the other legitimate one-sided derivative at a kink;
    `grid_mask`: per-scale [B,1,h,w] bool, pixels whose warp passes no gradient (synthesize).

    Note the reference's metric aliasing: `add_metric` stores `photometric_loss.detach()`
    (:296, loss_base.py:73-81) and `loss += smoothness` (:405) then adds IN PLACE into that
    same storage, so metrics['photometric_loss'] reports photometric + smoothness.
    """
    inv = [1.0 / (sigmoid_to_depth(s, min_depth, max_depth) + 1e-8) for s in sigs]
    n = num_scales(progressive_scaling, num_scales_, progress)
    H, W = image.shape[-2:]
    images = [resize_like(image, inv[i].shape) for i in range(n)]
    masks = [resize_like(mask, inv[i].shape, "nearest") for i in range(n)] if mask is not None else None

    def photo(ests, refs):
        out = []
        for i in range(n):
            p = photometric_map(ests[i], refs[i], ssim_loss_weight, C1, C2)
            if clip_loss > 0.0:
                p = torch.clamp(p, max=float(p.mean() + clip_loss * p.std()))
            if masks is not None:
                p = p * masks[i]
            out.append(p)
        return out

    cands = [[] for _ in range(n)]
    for ref, T in zip(contexts, pose_mats):
        refs = [resize_like(ref, inv[i].shape) for i in range(n)]
        warped = []
        for i in range(n):
            s = inv[i].shape[-1] / float(W)
            depth = 1.0 / inv[i].clamp(min=1e-6)          # utils/depth.py:103-120
            if isinstance(K, dict):
                sh = inv[i].shape[-2] / float(H)
                warped.append(synthesize(refs[i], depth, fisheye_scale(K, s, sh), fisheye_scale(ref_K, s, sh), T,
                                         kink_flip_eps, None if grid_mask is None else grid_mask[i]))
            else:
                warped.append(synthesize(refs[i], depth, scale_K(K, s), scale_K(ref_K, s), T, kink_flip_eps,
                                         None if grid_mask is None else grid_mask[i]))
        for i, p in enumerate(photo(warped, images)):
            cands[i].append(p)
        if automask_loss:
            for i, p in enumerate(photo(refs, images)):
                cands[i].append(p)

    reduced = []
    total = 0.0
    for i in range(n):                                     # :269-297
        if photometric_reduce_op == "mean":
            r = sum(c.mean() for c in cands[i]) / len(cands[i])
            reduced.append(None)
        elif tie_flip is not None:
            vals = torch.cat(cands[i], 1)
            order = vals.detach().sort(dim=1, stable=True)[1]          # first index first on exact ties
            pick = torch.where(tie_flip[i].to(vals.device), order[:, 1:2], order[:, 0:1])
            m = vals.gather(1, pick)
            reduced.append(m)
            r = m.mean()
        else:
            m = torch.cat(cands[i], 1).min(1, True)[0]
            reduced.append(m)
            r = m.mean()
        total = total + r
    photometric = total / n
    loss = photometric
    smooth = torch.zeros((), device=image.device)
    if smooth_loss_weight > 0.0:
        smooth = smooth_loss_weight * smoothness(sigs, images, n)
        loss = loss + smooth
    return loss.unsqueeze(0), loss.detach(), smooth, reduced


# ---------------------------------------------------------------------------------------------------------------------
# evaluation (Abs Rel gate)
# ---------------------------------------------------------------------------------------------------------------------
def depth_metrics(gt, pred, min_depth, max_depth, crop="garg", use_gt_scale=True):
    """[abs_rel, sq_rel, rmse, rmse_log, a1, a2, a3].  utils/depth.py:258-447 ('top-center' when shapes agree)."""
    B, _, H, W = gt.shape
    if pred.shape != gt.shape:
        full = torch.zeros_like(gt)
        top, left = H - pred.shape[2], (W - pred.shape[3]) // 2
        full[:, :, top:top + pred.shape[2], left:left + pred.shape[3]] = pred
        pred = full
    acc = torch.zeros(7, dtype=torch.float64)
    cm = None
    if crop == "garg":
        cm = torch.zeros(H, W, dtype=torch.bool)
        cm[int(0.40810811 * H):int(0.99189189 * H), int(0.03594771 * W):int(0.96405229 * W)] = True
    for b in range(B):
        g, p = gt[b, 0], pred[b, 0]
        valid = (g > min_depth) & (g < max_depth)
        if cm is not None:
            valid = valid & cm
        if valid.sum() == 0:
            continue
        g, p = g[valid], p[valid]
        if use_gt_scale:
            p = p * (torch.median(g) / torch.median(p))
        th = torch.max(g / p, p / g)
        d = g - p
        acc += torch.stack([(d.abs() / g).mean(), (d ** 2 / g).mean(), (d ** 2).mean().sqrt(),
                            ((g.log() - p.log()) ** 2).mean().sqrt(), (th < 1.25).float().mean(),
                            (th < 1.25 ** 2).float().mean(), (th < 1.25 ** 3).float().mean()]).double()
    return (acc / B).float()


# ---------------------------------------------------------------------------------------------------------------------
# test helpers: where is a fp32 implementation allowed to disagree with the reference's gradient?
# ---------------------------------------------------------------------------------------------------------------------
def sensitive_pixels(image, contexts, sigs, K, pose_mats, min_depth, max_depth, automask=True,
                     ssim_w=0.85, C1=1e-4, C2=9e-4, coord_eps=2e-4, margin_eps=5e-5, l1_eps=1e-4,
                     return_ties=False):
    """Per-scale boolean maps [B,1,h,w] of pixels whose gradient is discontinuous at fp32 precision:

    * bilinear kinks: a sampling coordinate within `coord_eps` px of an integer (2e-4: ~3 ulps of
      an fp32 pixel coordinate in [512, 1024), which passes through ~20 fp32 operations: lift,
      transform, project, normalise / un-normalise; 1e-4 let a real flip through in the rand_mask
      golden's pose gradient) — d(warp)/d(ix)
      jumps there (grid_sample's derivative is piecewise constant in the tap cell), so two fp32
      implementations that round ix to opposite sides get different gradients at that pixel;
    * min-reprojection near-ties: best and second-best candidate within `margin_eps` (fp32 SSIM
      carries ~1e-5 absolute error from the E[x^2]-mu^2 cancellation, so two fp32 implementations
      can order candidates differently below that) — the
      selected candidate (and so the gradient of the 3x3 SSIM window around it) can flip.
    * L1 sign near-ties: a warped value within `l1_eps` of the target in some channel (1e-4: a
      2e-4 px coordinate difference on a steep texture moves the warped value that much) — the
      derivative of |est - tgt| flips sign there (the selected candidate's 3x3 SSIM window aside,
      only that pixel's gradient moves).
    Computed in float64 from the same inputs.  A scale whose map is smaller than the image is
    evaluated as photometric_loss evaluates it (multi-resolution maps: the images resized to the
    map, the intrinsics scaled, :274-300).  With `return_ties` also the (undilated) near-tie maps,
    the `tie_flip` argument of photometric_loss.
    """
    out, ties = [], []
    fish = isinstance(K, dict)
    Kf = {k: v.double() for k, v in K.items()} if fish else K.double()
    mats = [m.double() for m in pose_mats]
    H0, W0 = image.shape[-2:]
    for s in sigs:
        s = s.double()
        H, W = s.shape[-2:]
        img = resize_like(image.double(), s.shape)
        ctx = [resize_like(c.double(), s.shape) for c in contexts]
        if (H, W) == (H0, W0):
            Kd = Kf
        else:
            Kd = fisheye_scale(Kf, W / float(W0), H / float(H0)) if fish else scale_K(Kf, W / float(W0))
        depth = 1.0 / (1.0 / (sigmoid_to_depth(s, min_depth, max_depth) + 1e-8)).clamp(min=1e-6)
        X = fisheye_lift(depth, Kd) if fish else lift(depth, Kd)
        bad = torch.zeros_like(s, dtype=torch.bool)
        cands = []
        for c, T in zip(ctx, mats):
            g = fisheye_project_to_grid(X, Kd, T) if fish else project_to_grid(X, Kd, T)
            ix = (g[..., 0] + 1) / 2 * (W - 1)
            iy = (g[..., 1] + 1) / 2 * (H - 1)
            kink = ((ix - ix.round()).abs() < coord_eps) | ((iy - iy.round()).abs() < coord_eps)
            bad |= kink.unsqueeze(1)
            warped = synthesize(c, depth, Kd, Kd, T)
            bad |= ((warped - img).abs() < l1_eps).any(1, keepdim=True)
            cands.append(photometric_map(warped, img, ssim_w, C1, C2))
            if automask:
                cands.append(photometric_map(c, img, ssim_w, C1, C2))
        tie = torch.zeros_like(s, dtype=torch.bool)
        if len(cands) > 1 and cands[0].shape[1] == 1:
            srt = torch.cat(cands, 1).sort(1)[0]
            tie = (srt[:, 1:2] - srt[:, 0:1]) < margin_eps
            # a flipped selection moves the gradient of the whole 3x3 SSIM window
            bad |= F.max_pool2d(tie.double(), 3, 1, 1) > 0
        out.append(bad)
        ties.append(tie)
    return (out, ties) if return_ties else out
