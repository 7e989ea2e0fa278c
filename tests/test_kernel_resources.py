"""CPU check of the built library's code-object metadata: the kernels the dispatcher launches
for the BASELINE configurations (and the quantised / MLA / GEMM rows beside them) use no
scratch memory, i.e. no register spills to HBM, and fit the register file.  A spill here is
silent on the GPU (results stay correct) and shows up only as extra HBM traffic in the
PMC passes; this pins it at build time.  Needs the ROCm LLVM tools (present
in this image); skipped otherwise."""
import os
import re
import shutil
import subprocess

import pytest

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_LIB = os.path.join(_REPO, "metal-flash-attention-plus_amd", "libmfa_amd.so")
_LLVM = "/opt/rocm/lib/llvm/bin"

# Mangled-name fragments of the tuned kernels (csrc/attention_fwd_v2.hip, attention_fwd_pipe.hip,
# attention_fwd_stream.hip,
# attention_fwd_i8.hip, attention_fwd_kv8.hip, attention_decode.hip, attention_bwd_fast.hip,
# attention_bigd.hip, attention_mla_latent.hip, kv_dequant.hip, gemm.hip, quantize.hip).
HOT = ("mfa_fwd2_kernel", "mfa_fwd2_pair_kernel", "mfa_fwd2_share_kernel", "mfa_fwd2_stream_kernel",
       "mfa_fwd_i8_kernel", "mfa_fwd2_kv8_kernel", "mfa_fwd_decode_kernel", "mfa_fwd_decode16_kernel", "mfa_decode_merge",
       "mfa_bwd_q_fast_kernel", "mfa_bwd_kv_fast_kernel", "mfa_fwd_bigd_kernel",
       "mfa_bwd_q_bigd_kernel", "mfa_mla", "mfa_kv_dequant_kernel", "mfa_gemm2_kernel",
       "mfa_gemm3_kernel", "qz_", "mfa_fwd_pipe_kernel", "mfa_fwd2_share_kv8_kernel")
# Known stack users, each a rare path, with a cap on what they may use (bytes of scratch per
# lane, spilled VGPRs) so that growth is caught:
# - the D > 256 backwardQuery with an FP32 dO (the quantised API's dO, DOS = SRC_F32ANY) keeps
#   160 B of its 64-register dO staging in scratch (no spill: vgpr_spill_count 0);
# - the D = 256 backwardKeyValue mask instantiation (additive masks / sparse ranges; the unmasked
#   D = 256 kernel sits exactly at 512 registers) spills 24 registers (52 B): it issues the next
#   step's tiles after its S/dP chains so the reloads never wait on them, and runs the masked
#   D = 256 backwardKeyValue 5.7x faster than the generic kernel it replaced (257 vs 1464 us,
#   B1 H16 S2048 additive mask).
EXEMPT = {"mfa_bwd_q_bigd_kernelINS_7Arith16INS_3F16ELi128EEELi128ELi3E": (160, 0),
          "mfa_bwd_q_bigd_kernelINS_7Arith16INS_4BF16ELi128EEELi128ELi3E": (160, 0),
          "mfa_bwd_kv_fast_kernelINS_3F16ELi256ELi32ELi0ELb1E": (64, 32),
          "mfa_bwd_kv_fast_kernelINS_4BF16ELi256ELi32ELi0ELb1E": (64, 32),
          # INT8 on-load forward at D = 256: three registers stored before the tile loop and
          # reloaded after it (none inside).
          "mfa_fwd2_kv8_kernelINS_3F16ELi256ELi32ELi1E": (16, 3),
          "mfa_fwd2_kv8_kernelINS_4BF16ELi256ELi32ELi1E": (16, 3)}


@pytest.fixture(scope="module")
def kernels(tmp_path_factory):
    if not (os.path.exists(_LIB) and os.path.exists(os.path.join(_LLVM, "llvm-readelf"))):
        pytest.skip("library or ROCm LLVM tools not present")
    d = tmp_path_factory.mktemp("co")
    lib = shutil.copy(_LIB, d)
    subprocess.run([os.path.join(_LLVM, "llvm-objdump"), "--offloading", lib], check=True,
                   capture_output=True, cwd=d)
    notes = ""
    for f in sorted(os.listdir(d)):
        if f.endswith("gfx950"):
            notes += subprocess.run([os.path.join(_LLVM, "llvm-readelf"), "--notes",
                                     os.path.join(d, f)], check=True, capture_output=True,
                                    text=True).stdout
    out = {}
    for ent in notes.split("- .agpr_count")[1:]:
        def field(k):
            m = re.search(r"\." + k + r":\s+(\S+)", ent)
            return m.group(1) if m else None
        out[field("name")] = {"scratch": int(field("private_segment_fixed_size")),
                              "vgpr_spill": int(field("vgpr_spill_count")),
                              "vgpr": int(field("vgpr_count"))}
    assert out, "no kernel metadata found"
    return out


def test_hot_kernels_present(kernels):
    for frag in HOT:
        assert any(frag in n for n in kernels), frag


def test_hot_kernels_use_no_scratch(kernels):
    bad = {n: k for n, k in kernels.items()
           if any(f in n for f in HOT) and k["scratch"] != 0 and not any(e in n for e in EXEMPT)}
    assert not bad, bad


def test_exempt_kernels_stay_within_caps(kernels):
    for frag, (max_scratch, max_spill) in EXEMPT.items():
        hits = {n: k for n, k in kernels.items() if frag in n}
        assert hits, frag
        for n, k in hits.items():
            assert k["scratch"] <= max_scratch and k["vgpr_spill"] <= max_spill, (n, k)


def test_hot_kernels_fit_register_file(kernels):
    for n, k in kernels.items():
        if any(f in n for f in HOT):
            assert k["vgpr"] <= 512, (n, k)


def test_generic_backward_kv_d256_does_not_spill(kernels):
    # The generic backwardKeyValue kernel (strided / transposed D = 256 16-bit calls) splits its
    # dK/dV columns over two workgroups (attention_bwd.h, DC = 128): no register spills (it spilled
    # ~470 before).  Its small fixed stack (no spill count) is the Stager's indexed staging.
    gen = {n: k for n, k in kernels.items()
           if "mfa_bwd_kv_kernel" in n and "Arith16" in n and "ELi256E" in n}
    assert gen, "generic D = 256 backwardKeyValue kernels not found"
    assert all(k["vgpr_spill"] == 0 for k in gen.values()), gen


def _design_kernel_table():
    """DESIGN.md §3's kernel table: the first cell of each row, and the section's whole text."""
    text = open(os.path.join(_REPO, "DESIGN.md")).read()
    sec = text[text.index("\n## 3."):text.index("\n## 4.")]
    first_cells = [ln.split("|")[1] for ln in sec.splitlines()
                   if ln.startswith("| `") and ln.count("|") >= 5]
    return first_cells, sec


def test_design_kernel_table_matches_library(kernels):
    # every kernel the DESIGN §3 table names exists in libmfa_amd.so, and every
    # kernel the library holds is named in DESIGN §3 (the table, or the section's text), so the
    # document cannot describe a deleted kernel or leave a shipped one out.
    cells, sec = _design_kernel_table()
    assert cells, "DESIGN §3 kernel table not found"
    named = set()
    for c in cells:
        for ident in re.findall(r"`((?:mfa|qz)_[A-Za-z0-9_]*)", c):
            named.add(ident)
    assert named, cells
    missing = sorted(n for n in named if not any(n in k for k in kernels))
    assert not missing, f"DESIGN §3 names kernels the library does not hold: {missing}"
    bases = set()
    for k in kernels:
        m = re.search(r"(mfa_[a-z0-9_]*?kernel|qz_[a-z0-9_]+?)(?:I|E|$|v$)", k)
        if m:
            bases.add(m.group(1))
    # (A name written as a prefix, e.g. `qz_absmax_*`, covers the kernels it starts.)
    undocumented = sorted(b for b in bases if b not in sec and not any(b.startswith(n) for n in named))
    assert not undocumented, f"library kernels not described in DESIGN §3: {undocumented}"
