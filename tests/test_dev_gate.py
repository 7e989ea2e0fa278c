"""The library's development A/B switches (MFA_FWD_SHARE, MFA_KV_REGS, MFA_GEMM3, ...) are read
only in a process started with MFA_DEV=1 (csrc/mfa_launch.h dev_env): a
production caller's environment must not change which kernel runs.  The plan query runs the
real dispatcher with launches recorded (no GPU), so a child process without MFA_DEV computes the
plans of the BASELINE shapes (C2, C3 fp16 / INT8, C5 forward and both backward phases, the
quantised backward) with no switch set and with every switch set, and they must be equal.  The
same child with MFA_DEV=1 must see the switches (else the check would be vacuous)."""
import json
import os
import subprocess
import sys

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# Every switch the dispatch path reads, with a value that changes a plan when MFA_DEV=1.
KNOBS = {
    "MFA_FWD_SHARE": "0", "MFA_FWD_VARIANT": "s", "MFA_FWD_PAIR": "o", "MFA_FWD_STREAM": "1",
    "MFA_FWD_STREAM_WGS": "7", "MFA_FWD_STREAM_SLOW": "1", "MFA_FWD_GEN": "1",
    "MFA_DISABLE_FAST": "1", "MFA_FWD2_TUNE": "1", "MFA_SHARE_XCD": "0", "MFA_SHARE_DV": "0",
    "MFA_SHARE_NT": "0", "MFA_SHARE_SWI": "0", "MFA_SHARE_IMG": "0", "MFA_KV8": "0",
    "MFA_BWDQ_BYTES": "1", "MFA_NO_DEQUANT_PASS": "1", "MFA_KV_REGS": "0", "MFA_DECODE": "0",
    "MFA_DECODE_MERGE": "1", "MFA_DECODE16": "0", "MFA_I8_BK": "1", "MFA_I8_SHARE": "0", "MFA_BWD256_BIGD": "1",
    "MFA_GEMM_IMG": "0", "MFA_GEMM_NN": "1", "MFA_GEMM3": "0",
}

_CHILD = r"""
import json, os, sys
sys.path.insert(0, os.path.join(sys.argv[1], "metal-flash-attention-plus_amd", "python"))
import mfa_amd as mfa
P, K = mfa.Precision, mfa.KernelType

def mh(B, H, S, D, causal=False):
    base = mfa.AttentionDescriptor.make(low_precision=True, precision=P.FP16, causal=causal)
    return mfa.MultiHeadDescriptor.make(base, B, H, S, D)

def names(plan):
    return [r["name"] for r in plan]

out = {}
out["C2"] = names(mfa.multihead_plan(mh(1, 16, 4096, 128, causal=True)))
out["C3"] = names(mfa.multihead_plan(mh(1, 16, 8192, 128)))
c5 = mh(8, 32, 4096, 256)
for k in (K.forward, K.backwardQuery, K.backwardKeyValue):
    out["C5-%d" % int(k)] = names(mfa.multihead_plan(c5, k))
base = mfa.AttentionDescriptor.make(8192, 8192, 128, low_precision=True, precision=P.FP16)
out["C3-int8"] = names(mfa.quantized_plan(mfa.quantized_descriptor(base, P.FP16, P.INT8, P.INT8, B=1, H=16)))
out["C3-i8mm"] = names(mfa.quantized_plan(
    mfa.quantized_descriptor(base, P.FP16, P.INT8, P.INT8, B=1, H=16, integer_matmul=True)))
b256 = mfa.AttentionDescriptor.make(4096, 4096, 256, low_precision=True, precision=P.FP16)
q256 = mfa.quantized_descriptor(b256, P.FP16, P.INT8, P.INT8, B=2, H=32)
for k in (K.forward, K.backwardQuery, K.backwardKeyValue):
    out["q256-%d" % int(k)] = names(mfa.quantized_plan(q256, k))
dec = mfa.AttentionDescriptor.make(1, 8192, 128, low_precision=True, precision=P.FP16)
out["decode"] = names(mfa.quantized_plan(mfa.quantized_descriptor(dec, P.FP16, P.INT8, P.INT8, B=32, H=16)))
out["decode-i4"] = names(mfa.quantized_plan(mfa.quantized_descriptor(dec, P.FP16, P.INT4, P.INT4, B=32, H=16)))
print(json.dumps(out))
"""


def _plans(env_extra):
    env = {k: v for k, v in os.environ.items() if not k.startswith("MFA_")}
    env.update(env_extra)
    r = subprocess.run([sys.executable, "-c", _CHILD, _REPO], env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_switches_do_not_change_plans_without_mfa_dev():
    plain = _plans({})
    knobbed = _plans(dict(KNOBS))
    assert knobbed == plain


def test_switches_are_seen_with_mfa_dev():
    plain = _plans({"MFA_DEV": "1"})
    knobbed = _plans(dict(KNOBS, MFA_DEV="1"))
    changed = [k for k in plain if plain[k] != knobbed[k]]
    assert "C2" in changed and "C3" in changed and "C3-int8" in changed, changed
