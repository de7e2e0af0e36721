"""Compare two gradient dumps of tools/train_dump.py (gpurun_out/g_base.npz vs gpurun_out/train_grads.npz): max |difference| per tensor."""
import numpy as np
a=np.load('gpurun_out/g_base.npz'); b=np.load('gpurun_out/train_grads.npz')
worst=0
for k in a.files:
    d=float(np.max(np.abs(a[k].astype(np.float64)-b[k]))) if a[k].size else 0.0
    worst=max(worst,d)
    if d: print(k, d)
print('max abs diff over', len(a.files), 'tensors:', worst)
