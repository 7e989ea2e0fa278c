"""Debug (development): block-wise on-load vs pass vs oracle on variants of one failing case."""
import os, sys
os.environ.setdefault("MFA_DEV", "1")
_REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(_REPO, "metal-flash-attention-plus_amd", "python"))
sys.path.insert(0, os.path.join(_REPO, "tests"))
import numpy as np, torch
import mfa_amd as mfa
import oracle_lib as ol
from harness import seen, to_device
P = mfa.Precision
DEV = "cuda:0"

def case(B, H, Hkv, R, C, D, bs, zp, qp, kv=P.INT8):
    rng = np.random.default_rng(R + C + D + bs)
    Q = rng.standard_normal((B, H, R, D)).astype(np.float32)
    kq = rng.integers(-120, 120, (B, Hkv, C, D)).astype(np.int8)
    vq = rng.integers(-120, 120, (B, Hkv, C, D)).astype(np.int8)
    rows = B * Hkv * C
    bcols = (D + bs - 1) // bs
    nb = ((rows + bs - 1) // bs) * bcols
    def blocks():
        s = rng.uniform(0.005, 0.03, nb).astype(np.float32)
        z = rng.integers(-3, 4, nb).astype(np.int32) if zp else np.zeros(nb, np.int32)
        return s, z
    (ks, kz), (vs, vz) = blocks(), blocks()
    bi = (np.arange(rows)[:, None] // bs) * bcols + np.arange(D)[None, :] // bs
    deq = lambda q, s, z: ((q.reshape(rows, D).astype(np.float32) - z[bi].astype(np.float32)) * s[bi]).astype(np.float32).reshape(B, Hkv, C, D)
    kd, vd = deq(kq, ks, kz), deq(vq, vs, vz)
    base = mfa.AttentionDescriptor.make(R, C, D, low_precision=True, precision=qp)
    desc = mfa.quantized_descriptor(base, qp, kv, kv, B=B, H=H, Hkv=Hkv)
    tq = mfa.quantized_tensor(to_device(Q, qp), qp)
    kt = torch.from_numpy(kq.view(np.uint8)).to(DEV); vt = torch.from_numpy(vq.view(np.uint8)).to(DEV)
    keep = [torch.from_numpy(x).to(DEV) for x in (ks, vs, kz, vz)]
    tk = mfa.QuantizedTensor(kt.data_ptr(), int(kv), 1.0, 0); tk.block_scales, tk.block_size = keep[0].data_ptr(), bs
    tv = mfa.QuantizedTensor(vt.data_ptr(), int(kv), 1.0, 0); tv.block_scales, tv.block_size = keep[1].data_ptr(), bs
    if zp: tk.block_zero_points, tv.block_zero_points = keep[2].data_ptr(), keep[3].data_ptr()
    def run():
        o = torch.full((B, H, R, D), float("nan"), dtype=torch.float32, device=DEV)
        l = torch.full((B, H, R), float("nan"), dtype=torch.float16, device=DEV)
        mfa.QuantizedAttention().forward(desc, tq, tk, tv, o, l); torch.cuda.synchronize()
        return o.cpu().numpy(), l.float().cpu().numpy()
    o1, l1 = run()
    os.environ["MFA_KV8_BW"] = "0"; os.environ["MFA_FWD_SHARE"] = "1"; o2, l2 = run(); os.environ.pop("MFA_KV8_BW"); os.environ.pop("MFA_FWD_SHARE")
    Qs = seen(Q, qp)
    e1 = e2 = 0.0
    for b in range(B):
        for h in range(H):
            ref = ol.attention(Qs[b:b+1, h:h+1], kd[b:b+1, h % Hkv:h % Hkv + 1], vd[b:b+1, h % Hkv:h % Hkv + 1])
            d1 = np.abs(o1[b:b+1, h:h+1] - ref["O"]).max(); d2 = np.abs(o2[b:b+1, h:h+1] - ref["O"]).max()
            e1, e2 = max(e1, d1), max(e2, d2)
            if d1 > 1e-2 or d2 > 1e-2: print(f"   b{b} h{h}: onload {d1:.3g} pass {d2:.3g}")
    diff = np.abs(o1 - o2)
    idx = np.argwhere(diff > 1e-6)
    print(f"B{B} H{H}/{Hkv} R{R} C{C} D{D} bs{bs} zp{zp} {qp}: onload err {e1:.3g} pass err {e2:.3g} equal {np.array_equal(o1, o2)} ndiff {len(idx)}",
          "first", idx[:3].tolist() if len(idx) else "", flush=True)

for args in [(2, 2, 2, 256, 777, 96, 48, True), (1, 2, 2, 256, 777, 96, 48, True), (2, 2, 2, 256, 777, 128, 48, True),
             (2, 2, 2, 256, 777, 128, 64, False), (1, 2, 2, 256, 777, 128, 64, False), (1, 4, 4, 512, 1000, 128, 64, False),
             (1, 2, 2, 256, 768, 128, 64, False), (1, 2, 2, 512, 777, 128, 64, False)]:
    case(*args, P.FP16)
