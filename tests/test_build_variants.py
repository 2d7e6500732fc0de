"""Every compile-time knob the kernel sources keep (rr_kernels.hip, rr_decode_class.h,
rr_snappy.hip) still compiles for gfx950 with a non-default value, so no kept path rots: a
front-end pass (templates instantiated, static_asserts checked) of each variant's device code.
The default build is compiled in full by __graft_entry__.build().  CPU only (hipcc
cross-compiles); skipped where hipcc is absent."""
import os
import re
import shutil
import subprocess

import pytest

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "redrock_old_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"

# (source, -D flags): one non-default setting per kept knob
VARIANTS = [
    ("rr_kernels.hip", "-DRR_PROBE"),
    ("rr_kernels.hip", "-DRR_ABLATE=1"),
    ("rr_kernels.hip", "-DRR_ABLATE=2"),
    ("rr_kernels.hip", "-DRR_ABLATE=3"),
    ("rr_kernels.hip", "-DRR_ABLATE=4"),
    ("rr_kernels.hip", "-DRR_ABLATE=5"),
    ("rr_kernels.hip", "-DRR_ABLATE=6"),
    ("rr_kernels.hip", "-DRR_DEC_W=65536"),
    ("rr_kernels.hip", "-DRR_DEC_SLACK=8192"),
    ("rr_kernels.hip", "-DRR_DEC_NW=4"),
    ("rr_kernels.hip", "-DRR_ZL_VPB=8 -DRR_HH_VPB=16 -DRR_HT_VPB=8 -DRR_LIST_VPB=8"),
    ("rr_kernels.hip", "-DRR_ENC_W=8192 -DRR_ENC_RCAP=256"),
    ("rr_snappy.hip", "-DRR_SNZ_DEC_WIN=16384"),
    ("rr_snappy.hip", "-DRR_SNZ_FRAG=16448"),
    ("rr_snappy.hip", "-DRR_SNZ_K=1"),
    ("rr_snappy.hip", "-DRR_SNZ_K=32"),
    ("rr_snappy.hip", "-DRR_SNZ_SPEC=0"),
    ("rr_snappy.hip", "-DRR_SNZ_SPARSE=4096"),
    ("rr_snappy.hip", "-DRR_SNZ_SPARSE=2048 -DRR_SNZ_K=1"),
    ("rr_snappy.hip", "-DRR_PROBE"),
]


def _knobs(src):
    with open(os.path.join(CSRC, src)) as f:
        text = f.read()
    return set(re.findall(r"^\s*#\s*(?:if|ifdef|ifndef|elif)\b.*?\b(RR_[A-Z0-9_]+)", text, re.M)) - {
        "RR_INTERNAL_H", "RR_KERNELS_H"}


def test_every_knob_has_a_variant():
    """The variant list covers every RR_* knob the sources test (and they stay few)."""
    knobs = _knobs("rr_kernels.hip") | _knobs("rr_decode_class.h") | _knobs("rr_snappy.hip")
    covered = set(re.findall(r"-D(RR_[A-Z0-9_]+)", " ".join(f for _, f in VARIANTS)))
    assert knobs <= covered, sorted(knobs - covered)
    assert len(knobs) <= 16, sorted(knobs)


@pytest.mark.skipif(not os.path.exists(HIPCC) or shutil.which("clang") is None and not os.path.exists(HIPCC),
                    reason="hipcc not installed")
@pytest.mark.parametrize("src,flags", VARIANTS, ids=[f"{s}:{f}" for s, f in VARIANTS])
def test_variant_compiles(src, flags):
    cmd = [HIPCC, "--offload-arch=gfx950", "-std=c++17", "--cuda-device-only", "-fsyntax-only", "-Wno-unused-command-line-argument",
           *flags.split(), src]
    r = subprocess.run(cmd, cwd=CSRC, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
