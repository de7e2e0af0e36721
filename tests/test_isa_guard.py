"""ISA guard (CPU): no kernel of libavse.so may contain `v_pk_add_f32` with an op_sel modifier.

On gfx950 `v_pk_add_f32` with a half-swapping op_sel on its second source returned wrong values in lanes 48..63 when
another kernel's MFMA work shared the CU (round 5: tools/pk_probe.py); the STFT helpers that used it
are now v_pk_fma forms and the ISTFT is built without SLP pairing (which generated the same form).  This test
disassembles the gfx950 code objects of the built objects (audio-visual-speech-enhancement_amd/csrc/build/*.o, the
library's own) and fails on any `v_pk_add_f32 ... op_sel:` — forms the hardware probe has not cleared."""
import glob
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "audio-visual-speech-enhancement_amd", "csrc", "build")
LLVM = "/opt/rocm/lib/llvm/bin"
BAD = re.compile(r"v_pk_add_f32\s.*\bop_sel:")


def _disassemble(obj, tmp):
    fat = os.path.join(tmp, os.path.basename(obj) + ".fatbin")
    co = os.path.join(tmp, os.path.basename(obj) + ".co")
    r = subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj], capture_output=True, text=True)
    if r.returncode != 0 and "not found" in r.stderr:
        return ""   # a host-only object (no device code)
    r.check_returncode()
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                    f"--input={fat}", f"--output={co}", "--unbundle"], check=True, capture_output=True)
    return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], check=True, capture_output=True,
                          text=True).stdout


def test_no_op_sel_packed_adds(tmp_path):
    objs = sorted(glob.glob(os.path.join(BUILD, "*.o")))
    if not objs or not os.path.exists(f"{LLVM}/clang-offload-bundler"):
        pytest.skip("no built objects / ROCm LLVM tools (run __graft_entry__.build())")
    found = {}
    for obj in objs:
        bad = [line.strip() for line in _disassemble(obj, str(tmp_path)).splitlines() if BAD.search(line)]
        if bad:
            found[os.path.basename(obj)] = (len(bad), bad[:2])
    assert not found, f"v_pk_add_f32 with op_sel in: {found}"
