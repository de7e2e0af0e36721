"""Diagnostic: a packed-FP32 VALU chain (tools/pk_probe.hip k_pk_victim) run alone and beside matrix-core work on a
second stream; prints how many runs and which lanes differ from the solo result (kind 0 v_pk_fma_f32, 1 v_fma_f32).
    python tools/pk_probe.py [reps]
"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from isa_forms import PROBE_FORMS   # noqa: E402  (kind -> (mnemonic, modifiers); the ISA guard's allow-list)

NAMES = {0: 'v_pk_fma_f32', 1: 'v_fma_f32', 2: 'LDS round trip + v_pk_fma_f32', 3: 'STFT op_sel packed helpers',
         4: 'pk_fma op_sel+neg (pk_cmul_t)', 5: 'pk_add op_sel+neg (pk_add_mi)', 6: 'pk_add neg only (pk_sub_conj)',
         7: 'pk_add op_sel only', 8: 'pk_add_mi / pk_sub_mi as v_pk_fma (round 5)'}
NAMES.update({k: f"{mn} {mod}" for k, (mn, mod) in PROBE_FORMS.items()})


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "_stress", "libpk_probe.so"))
    dev = torch.device("cuda", 0)
    s0, s1 = torch.cuda.current_stream(dev), torch.cuda.Stream(dev)
    blocks, iters = 1024, 4000
    inp = torch.rand(4096, device=dev)
    busy = torch.empty(8192 * 256, device=dev)
    for kind in [int(k) for k in os.environ.get('PK_KINDS', '3,4,5,6,7,0').split(',')]:
        ref = torch.empty(blocks * 448 * 2, device=dev)
        lib.pk_victim(kind, ctypes.c_void_p(inp.data_ptr()), ctypes.c_void_p(ref.data_ptr()), blocks, iters,
                      ctypes.c_void_p(s0.cuda_stream))
        torch.cuda.synchronize()
        for mode in ("solo", "beside MFMA"):
            nbad, lanes, elems = 0, set(), 0
            for _ in range(reps):
                out = torch.empty_like(ref)
                if mode != "solo":
                    lib.mfma_busy(int(mode.endswith("LDS")), ctypes.c_void_p(busy.data_ptr()), 8192, 20000,
                                  ctypes.c_void_p(s1.cuda_stream))
                lib.pk_victim(kind, ctypes.c_void_p(inp.data_ptr()), ctypes.c_void_p(out.data_ptr()), blocks, iters,
                              ctypes.c_void_p(s0.cuda_stream))
                torch.cuda.synchronize()
                diff = (out != ref).view(blocks * 448, 2).any(dim=1)
                if diff.any():
                    nbad += 1
                    idx = diff.nonzero().flatten()
                    elems += idx.numel()
                    lanes |= set((idx % 64).tolist())
            print(f"kind {kind} ({NAMES.get(kind, '?')}) {mode}: {nbad} of {reps} runs differ "
                  f"({elems} threads); lanes {sorted(lanes)[:16]}{' ...' if len(lanes) > 16 else ''} "
                  f"({len([l for l in lanes if l >= 32])} of {len(lanes)} in 32..63)", flush=True)


if __name__ == "__main__":
    main()
