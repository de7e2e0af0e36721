"""CPU property tests of host logic and of the index arithmetic the HIP transforms are built on.

* `shard_bounds` (parallel.py) partitions any clip / utterance count over any world size into contiguous blocks whose
  sizes differ by at most one (the bench's and `sharded_predict`'s sharding).
* `ops.n_frames` equals the number of centred frame starts librosa.stft produces (data_processor.py:44-50 geometry).
* The Good-Thomas index maps compiled into `k_spec533` (stft.hip: n = (41 n1 + 13 n2) mod 533, k = (287 k1 + 247 k2)
  mod 533) and `k_istft532` (istft.hip: k = (19 k1 + 28 k2) mod 532, n = (57 n1 + 476 n2) mod 532) are bijections that
  turn the 533-point DFT / 532-point inverse into 13 x 41 / 28 x 19 two-dimensional transforms with no twiddles, and the
  Hermitian fold k_istft532 uses (Z[28 - k1][n2] = conj Z[k1][n2]) holds: checked against numpy's FFT in float64.
"""
import numpy as np
from hypothesis import given, settings, strategies as st

from avse_amd.ops import n_frames
from avse_amd.parallel import shard_bounds


@settings(max_examples=300, deadline=None)
@given(n=st.integers(0, 100_000), world=st.integers(1, 64))
def test_shard_bounds_partition(n, world):
    blocks = [shard_bounds(n, world, r) for r in range(world)]
    assert blocks[0][0] == 0 and blocks[-1][1] == n
    for (a, b), (c, _) in zip(blocks, blocks[1:]):
        assert b == c
    sizes = [b - a for a, b in blocks]
    assert min(sizes) >= 0 and max(sizes) - min(sizes) <= 1
    assert sizes == sorted(sizes, reverse=True)   # the remainder goes to the lowest ranks


@settings(max_examples=200, deadline=None)
@given(L=st.integers(1, 60_000), n_fft=st.sampled_from([533, 640, 1024]), hop_div=st.sampled_from([4]))
def test_n_frames_counts_centred_frame_starts(L, n_fft, hop_div):
    hop = n_fft // hop_div
    padded = L + 2 * (n_fft // 2)
    starts = range(0, padded - n_fft + 1, hop)
    assert n_frames(L, hop, n_fft) == len(starts)


def _crt_maps(N, N1, N2, in_a, in_b, out_a, out_b):
    n = np.array([[(in_a * i + in_b * j) % N for j in range(N2)] for i in range(N1)])
    k = np.array([[(out_a * i + out_b * j) % N for j in range(N2)] for i in range(N1)])
    return n, k


def test_pfa533_maps_give_the_dft():
    n, k = _crt_maps(533, 13, 41, 41, 13, 287, 247)
    assert sorted(n.ravel()) == list(range(533)) and sorted(k.ravel()) == list(range(533))
    rng = np.random.default_rng(533)
    x = rng.standard_normal(533)                       # k_spec533's input: one real windowed frame
    X = np.fft.fft(x)
    # 41-point DFTs along n2 for each n1, then 13-point DFTs along n1 (no twiddle factors between the stages)
    Y = np.fft.fft(np.fft.fft(x[n], axis=1), axis=0)
    np.testing.assert_allclose(Y, X[k], rtol=0, atol=1e-10 * np.abs(X).max())


def test_pfa532_inverse_maps_and_hermitian_fold():
    n, _ = _crt_maps(532, 28, 19, 57, 476, 0, 0)
    k, _ = _crt_maps(532, 28, 19, 19, 28, 0, 0)
    assert sorted(n.ravel()) == list(range(532)) and sorted(k.ravel()) == list(range(532))
    rng = np.random.default_rng(532)
    X = np.fft.rfft(rng.standard_normal(532))          # 267 bins, as librosa.istft receives for n_fft 533
    full = np.concatenate([X, np.conj(X[-2:0:-1])])    # the Hermitian spectrum the 532-point inverse sees
    x = np.fft.ifft(full).real * 532                   # unnormalised inverse, like the kernel before its window scale
    # stage A: 19-point inverse DFTs along k2 for each k1; the fold k_istft532 relies on
    Z = np.fft.ifft(full[k], axis=1) * 19
    np.testing.assert_allclose(Z[(28 - np.arange(28)) % 28], np.conj(Z), atol=1e-9 * np.abs(Z).max())
    # stage B: 28-point inverse DFTs along k1; the output map puts sample n = (57 n1 + 476 n2) mod 532 at [n1, n2]
    Y = np.fft.ifft(Z, axis=0) * 28
    np.testing.assert_allclose(Y.real, x[n], rtol=0, atol=1e-9 * np.abs(x).max())
    np.testing.assert_allclose(Y.imag, 0, atol=1e-9 * np.abs(x).max())
