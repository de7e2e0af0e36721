"""Host side of SpeechEnhancementNetwork.train (network.py:177-206): the Keras 2.0 callback rules restated in
fit.py, and self-checks of the training oracle (oracle/keras_train_ref.py).  CPU only."""
import numpy as np
import pytest
import torch

from oracle import keras_train_ref as KT


def test_reduce_lr_on_plateau_keras_2_0_rule():
    from avse_amd.fit import ReduceLROnPlateau
    cb = ReduceLROnPlateau(factor=0.5, patience=5, min_lr=0)
    lr, lrs = 1.0, []
    # improves twice, then stalls: Keras halves after the 6th non-improving epoch (wait reaches 5 first)
    for v in [1.0, 0.9] + [0.9] * 13:
        lr = cb.on_epoch_end(v, lr)
        lrs.append(lr)
    assert lrs[:7] == [1.0] * 7
    assert lrs[7] == 0.5
    assert lrs[13] == 0.25
    # an improvement smaller than epsilon (1e-4) does not count
    cb = ReduceLROnPlateau(patience=0)
    assert cb.on_epoch_end(1.0, 1.0) == 1.0
    assert cb.on_epoch_end(1.0 - 5e-5, 1.0) == 0.5
    # at min_lr the rate is not reduced and the wait is NOT restarted (keras/callbacks.py 2.0.x: `self.wait = 0` sits
    # inside the `old_lr > min_lr + lr_epsilon` branch)
    cb = ReduceLROnPlateau(factor=0.5, patience=2, min_lr=0.25)
    lr, waits = 0.5, []
    for v in [1.0] + [1.0] * 8:
        lr = cb.on_epoch_end(v, lr)
        waits.append(cb.wait)
    assert lr == 0.25
    assert waits == [0, 1, 2, 1, 2, 3, 4, 5, 6]


def test_early_stopping_keras_2_0_rule():
    from avse_amd.fit import EarlyStopping
    cb = EarlyStopping(min_delta=0.01, patience=10)
    stops = [cb.on_epoch_end(v) for v in [1.0] + [0.995] * 12]
    # 0.995 is not an improvement of more than 0.01: the stop comes on the 11th non-improving epoch
    assert stops.index(True) == 11


def test_dropout_mask_is_deterministic_and_keeps_three_quarters():
    m1 = KT.dropout_scale(7, 5, (2, 64, 64, 128), 0.25)
    m2 = KT.dropout_scale(7, 5, (2, 64, 64, 128), 0.25)
    m3 = KT.dropout_scale(8, 5, (2, 64, 64, 128), 0.25)
    assert np.array_equal(m1, m2) and not np.array_equal(m1, m3)
    assert set(np.unique(m1)) == {0.0, 1.0 / 0.75}
    assert abs(np.mean(m1 > 0) - 0.75) < 0.005


def test_oracle_batchnorm_uses_batch_statistics():
    x = torch.randn(6, 3, 4, 4, dtype=torch.float64) * 3 + 2
    stats = {}
    y = KT._bn_train(x, torch.ones(3, dtype=torch.float64), torch.zeros(3, dtype=torch.float64), 1, stats, "l")
    assert torch.allclose(y.mean(dim=(0, 2, 3)), torch.zeros(3, dtype=torch.float64), atol=1e-12)
    var = y.var(dim=(0, 2, 3), unbiased=False)
    # (x - mu) / sqrt(var + 1e-3): slightly under unit variance
    assert torch.allclose(var, torch.as_tensor(stats["l"][1]) / (torch.as_tensor(stats["l"][1]) + 1e-3))


def test_oracle_adam_first_step_is_lr_sign():
    p = {"w/kernel": np.array([1.0, -2.0, 3.0])}
    g = {"w/kernel": np.array([0.5, -0.1, 2.0])}
    m = {"w/kernel": np.zeros(3)}
    v = {"w/kernel": np.zeros(3)}
    KT.adam_step(p, g, m, v, t=1, lr=1e-3)
    # first Keras Adam step: lr * sqrt(1 - b2) / (1 - b1) * (0.1 g) / (sqrt(0.001 g^2) + eps) = lr * sign(g)
    np.testing.assert_allclose(p["w/kernel"], [1.0 - 1e-3, -2.0 + 1e-3, 3.0 - 1e-3], rtol=1e-7)


@pytest.mark.parametrize("bad", [(80, 24)])
def test_trainer_python_api_checks_shapes(bad):
    from avse_amd import ops
    with pytest.raises(Exception):
        ops._dev_f32(torch.zeros((2,) + bad), "audio", (80, 20))
