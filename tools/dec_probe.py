import sys, torch
sys.path.insert(0, "metal-flash-attention-plus_amd/python")
import mfa_amd as mfa
P = mfa.Precision
B, H, Sq, Skv, D, lat = 32, 16, 1, 4096, 128, 512
bf = torch.bfloat16
latent = torch.randn(B * Skv, lat, device="cuda").to(bf)
wk = (torch.randn(lat, H * D, device="cuda") * lat ** -0.5).to(bf)
wv = (torch.randn(lat, H * D, device="cuda") * lat ** -0.5).to(bf)
q = torch.randn(B, H, Sq, D, device="cuda").to(bf)
o = torch.empty(B, H, Sq, D, device="cuda")
base = mfa.AttentionDescriptor.make(low_precision=True, precision=P.BF16)
for _ in range(20):
    mfa.mla_forward_absorbed(base, latent, wk, wv, q, o, B, H, Sq, Skv, D, lat, P.BF16)
torch.cuda.synchronize()
