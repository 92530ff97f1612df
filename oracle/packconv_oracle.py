"""ORACLE — test infrastructure only (never imported by the product path).

The composed PackNet packing layer (include/psfm_packconv.h) restated with torch ops:
  * `chain`  — the reference's own op chain, packnet_sfm/networks/layers/packnet/layers01.py:239-246
    (packing :126-146 -> Conv3d(1 -> d, 3x3x3, pad 1) -> view) and Conv2D's ConstantPad2d + Conv2d
    (:34-39): the oracle every parity test compares with;
  * `compose` — the composition the HIP kernels compute (k_pc_comp_*): Weff, the edge-line and corner
    weights and the bias3 table, in the reference's packed-channel order;
  * `kernel_layouts` — the same tensors in the kernel layouts of psfm_pc_weights (for decoding /
    checking the HIP composer);
  * `composed_forward` — the decomposition y = conv(P, Weff) + BT - edges + corners with torch ops.
tests/test_packconv.py proves, in float64 on the CPU, that `composed_forward` equals `chain` for y
and every gradient (the identity the kernels rely on).
"""
import torch
import torch.nn.functional as F


def packing(x, r=2):
    """layers01.py:126-146: [B,C,H,W] -> [B,C r^2,H/r,W/r], channel 4 c + 2 i + j."""
    b, c, h, w = x.shape
    x = x.contiguous().view(b, c, h // r, r, w // r, r)
    return x.permute(0, 1, 3, 5, 2, 4).reshape(b, c * r * r, h // r, w // r)


def chain(x, W2, w3, b3, k):
    """PackLayerConv3d.forward up to the Conv2d (no Conv2d bias): layers01.py:239-246 + :34-39."""
    V = F.conv3d(packing(x).unsqueeze(1), w3, b3, padding=1)
    B, d, Kp, Ho, Wo = V.shape
    return F.conv2d(F.pad(V.reshape(B, d * Kp, Ho, Wo), [k // 2] * 4), W2)


def class_masks(k, dtype, device):
    """[2pk+1, k]: tap i of the Conv2d is inside the image for output rows of class rc (rows
    0..pk-1, the interior, rows H-pk..H-1; the same for columns)."""
    pk = k // 2
    rc = torch.arange(2 * pk + 1, device=device)[:, None]
    i = torch.arange(k, device=device)[None, :]
    return ((i >= (pk - rc).clamp(min=0)) & (i <= (3 * pk - rc).clamp(max=k - 1))).to(dtype)


def compose(W2, w3, b3, k):
    """Composed weights in the reference's packed-channel order kp = 4 c + s:
        Weff   [C, 4C, k+2, k+2]
        U      [4 (T, B, L, R), pk, C, 4C, k+2]   edge line e of each side
        corner [4 (TL, BL, TR, BR), pk, pk, C, 4C]
        bt     [2pk+1, 2pk+1, C]
    T: U[0][e] is tap row i = e of W2 composed with w3's dy = 2 plane (output row Y = pk-1-e
    reads P's row 0); B: i = pk+1+e with dy = 0 (row Ho-1-e, P row Ho-1); L / R the same for
    columns.  Corner (i, j) of TL composes W2[.., i, j] with w3[.., 2, 2] (output pixel
    (pk-1-i, pk-1-j), P pixel (0, 0)); BL / TR / BR mirror it."""
    C, d = W2.shape[0], w3.shape[0]
    Kp, pk = W2.shape[1] // d, k // 2
    W2r = W2.reshape(C, d, Kp, k, k)
    Weff = F.conv_transpose3d(W2r, w3, padding=(1, 0, 0)).reshape(C, Kp, k + 2, k + 2)

    def rows(i0, i1, dy):
        Wi = W2r[:, :, :, i0:i1, :].permute(3, 0, 1, 2, 4).reshape(-1, d, Kp, 1, k)
        return F.conv_transpose3d(Wi, w3[:, :, :, dy:dy + 1, :], padding=(1, 0, 0)).reshape(i1 - i0, C, Kp, k + 2)

    def cols(j0, j1, dx):
        Wj = W2r[:, :, :, :, j0:j1].permute(4, 0, 1, 2, 3).reshape(-1, d, Kp, k, 1)
        return F.conv_transpose3d(Wj, w3[:, :, :, :, dx:dx + 1], padding=(1, 0, 0)).reshape(j1 - j0, C, Kp, k + 2)

    def corner(i0, i1, j0, j1, dy, dx):
        Wc = W2r[:, :, :, i0:i1, j0:j1].permute(3, 4, 0, 1, 2).reshape(-1, d, Kp, 1, 1)
        u = F.conv_transpose3d(Wc, w3[:, :, :, dy:dy + 1, dx:dx + 1], padding=(1, 0, 0))
        return u.reshape(i1 - i0, j1 - j0, C, Kp)

    U = torch.stack([rows(0, pk, 2), rows(pk + 1, k, 0), cols(0, pk, 2), cols(pk + 1, k, 0)])
    Cn = torch.stack([corner(0, pk, 0, pk, 2, 2), corner(pk + 1, k, 0, pk, 0, 2),
                      corner(0, pk, pk + 1, k, 2, 0), corner(pk + 1, k, pk + 1, k, 0, 0)])
    Bs = torch.einsum("mokij,o->mij", W2r, b3)
    M = class_masks(k, W2.dtype, W2.device)
    bt = torch.einsum("mij,ri,cj->rcm", Bs, M, M)
    return Weff, U, Cn, bt


def kin_order(t, C, dim):
    """Reference packed channel kp = 4 c + s -> kernel order kin = s C + c along `dim`."""
    dim = dim % t.dim()
    sh = list(t.shape)
    return t.reshape(sh[:dim] + [C, 4] + sh[dim + 1:]).transpose(dim, dim + 1).reshape(sh)


def ref_order(t, C, dim):
    """kin = s C + c -> reference kp = 4 c + s along `dim`."""
    dim = dim % t.dim()
    sh = list(t.shape)
    return t.reshape(sh[:dim] + [4, C] + sh[dim + 1:]).transpose(dim, dim + 1).reshape(sh)


def pad_rows(t, n):
    return t if t.shape[0] == n else torch.cat([t, t.new_zeros((n - t.shape[0],) + tuple(t.shape[1:]))])


def cop(n):
    return (n + 63) // 64 * 64


def kernel_layouts(Weff, U, Cn, bt, C, k):
    """The kernel layouts of include/psfm_packconv.h (bf16 weights, fp32 corner / bias tables)."""
    ke, pk = k + 2, k // 2
    bf = torch.bfloat16
    Wk = kin_order(Weff, C, 1)                                                      # [m][kin][a][b]
    wf = pad_rows(Wk, cop(C)).reshape(cop(C) // 64, 64, C // 8, 4, 8, ke, ke)
    wf = wf.permute(0, 2, 5, 6, 3, 1, 4).contiguous().to(bf)
    wb = Wk.flip(2, 3).reshape(C // 32, 4, 8, 4 * C // 64, 64, ke, ke)
    wb = wb.permute(3, 0, 5, 6, 1, 4, 2).contiguous().to(bf)
    Uk = kin_order(U, C, 3).reshape(4, pk * C, 4 * C, ke)                           # [edge][(e, m)][kin][s]
    ef = [pad_rows(Uk[e], cop(pk * C)).reshape(cop(pk * C) // 64, 64, C // 8, 4, 8, ke)
          .permute(0, 2, 5, 3, 1, 4).contiguous().to(bf) for e in range(4)]
    eb = [Uk[e].flip(2).reshape(pk * C // 32, 4, 8, 4 * C // 64, 64, ke)
          .permute(3, 0, 5, 1, 4, 2).contiguous().to(bf) for e in range(4)]
    corner = kin_order(Cn, C, 4).float().contiguous()
    return wf, wb, ef, eb, corner, bt.float().contiguous()




def composed_forward(x, W2, w3, b3, k):
    """The kernels' decomposition written with torch ops on `compose`'s tensors."""
    C = W2.shape[0]
    pk, pe, ke = k // 2, k // 2 + 1, k + 2
    P = packing(x)
    B, Kp, Ho, Wo = P.shape
    Weff, U, Cn, bt = compose(W2, w3, b3, k)
    y = F.conv2d(P, Weff, padding=pe)
    rc = lambda n: torch.tensor([i if i < pk else (2 * pk - (n - 1 - i) if i >= n - pk else pk) for i in range(n)])
    y = y + bt[rc(Ho)][:, rc(Wo)].permute(2, 0, 1)
    lines = [P[:, :, 0, :], P[:, :, Ho - 1, :], P[:, :, :, 0], P[:, :, :, Wo - 1]]
    E = [F.conv1d(l_, U[e].reshape(pk * C, Kp, ke), padding=pe).reshape(B, pk, C, -1) for e, l_ in enumerate(lines)]
    corr = torch.zeros_like(y)
    corr[:, :, :pk, :] += E[0].flip(1).permute(0, 2, 1, 3)
    corr[:, :, Ho - pk:, :] += E[1].flip(1).permute(0, 2, 1, 3)
    corr[:, :, :, :pk] += E[2].flip(1).permute(0, 2, 3, 1)
    corr[:, :, :, Wo - pk:] += E[3].flip(1).permute(0, 2, 3, 1)
    # corners: TL (i, j) -> pixel (pk-1-i, pk-1-j) from P[0, 0]; BL -> (Ho-1-i, pk-1-j); TR; BR:
    # (i, j) runs backwards through each pk x pk block
    px = [P[:, :, 0, 0], P[:, :, Ho - 1, 0], P[:, :, 0, Wo - 1], P[:, :, Ho - 1, Wo - 1]]
    cf = torch.zeros_like(y)
    for cn in range(4):
        v = torch.einsum("ijmk,bk->bmij", Cn[cn], px[cn]).flip(2, 3)
        ys = slice(0, pk) if cn % 2 == 0 else slice(Ho - pk, Ho)
        xs = slice(0, pk) if cn < 2 else slice(Wo - pk, Wo)
        cf[:, :, ys, xs] = cf[:, :, ys, xs] + v
    return y - corr + cf
