"""Keras-2.0 `Model.fit` loop of SpeechEnhancementNetwork.train (/root/reference/network.py:177-206) over libavse's
training step (ops.Trainer, csrc/train.hip).

The reference calls `fit(batch_size=16, epochs=1000, validation_data=..., callbacks=[ModelCheckpoint(path),
ReduceLROnPlateau('val_loss', factor=0.5, patience=5, min_lr=0), EarlyStopping('val_loss', min_delta=0.01,
patience=10), TensorBoard(...)])`.  Restated here (Keras 2.0.x callbacks.py semantics):
  * every epoch: shuffle the training set, one Adam step per batch of 16 (the last batch may be smaller), then
    val_loss = mean squared error of the validation set in inference mode (moving BN statistics, no dropout);
  * ModelCheckpoint: save the model after every epoch (save_best_only=False);
  * ReduceLROnPlateau: an epoch improves when val_loss < best - 1e-4; after `patience` further epochs without one,
    lr <- max(lr * 0.5, min_lr) and the wait restarts;
  * EarlyStopping: an epoch improves when val_loss + min_delta < best; training stops once the wait counter has
    reached `patience` on a non-improving epoch;
  * TensorBoard: not reproduced (no TensorFlow); the per-epoch history is returned instead.
The whole training and validation set is uploaded to HBM once (288 GB per MI355X), batches are gathered on device.
"""
import numpy as np
import torch

from . import ops


class ReduceLROnPlateau:
    """keras.callbacks.ReduceLROnPlateau (2.0.x), mode 'min', epsilon 1e-4, cooldown 0."""

    def __init__(self, factor=0.5, patience=5, min_lr=0.0, epsilon=1e-4):
        self.factor, self.patience, self.min_lr, self.epsilon = factor, patience, min_lr, epsilon
        self.best, self.wait = np.inf, 0

    def on_epoch_end(self, current, lr):
        if current < self.best - self.epsilon:
            self.best, self.wait = current, 0
        else:
            if self.wait >= self.patience:
                # keras/callbacks.py 2.0.x: the wait restarts only when the rate was actually reduced
                if lr > self.min_lr + 1e-4 * self.min_lr:
                    lr = max(lr * self.factor, self.min_lr)
                    self.wait = 0
            self.wait += 1
        return lr


class EarlyStopping:
    """keras.callbacks.EarlyStopping (2.0.x), mode 'min'."""

    def __init__(self, min_delta=0.01, patience=10):
        self.min_delta, self.patience = abs(min_delta), patience
        self.best, self.wait, self.stop = np.inf, 0, False

    def on_epoch_end(self, current):
        if current + self.min_delta < self.best:
            self.best, self.wait = current, 0
        else:
            if self.wait >= self.patience:
                self.stop = True
            self.wait += 1
        return self.stop


def _device(x, device):
    t = x if isinstance(x, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32))
    return t.to(device=device, dtype=torch.float32).contiguous()


def validation_loss(model, mixed, video, speech, batch=256):
    """Model.evaluate on the validation set: inference-mode MSE over every element (ops.forward, fp32)."""
    dw = ops.DeviceWeights(model, "float32", mixed.device)
    total, n = 0.0, mixed.shape[0]
    for a in range(0, n, batch):
        b = min(n, a + batch)
        pred = ops.forward(dw, mixed[a:b], video[a:b])
        total += float(ops.mse(pred, speech[a:b]).item()) * (b - a)
    return total / max(n, 1)


def fit(model, train, validation, model_cache_path=None, batch_size=16, epochs=1000, lr=5e-4, dropout=0.25,
        seed=0, device=None, verbose=1, save=None):
    """train / validation: (mixed [N, 80, 20], video [N, 128, 128, 5] (normalised), speech [N, 80, 20]).
    Returns (final KerasModel, history = [{'epoch', 'loss', 'val_loss', 'lr'}])."""
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    tm, tv, ts = (_device(x, dev) for x in train)
    vm, vv, vs = (_device(x, dev) for x in validation)
    n = tm.shape[0]
    trainer = ops.Trainer(model, max_batch=batch_size, device=dev)
    rng = np.random.default_rng(seed)
    plateau, stopper = ReduceLROnPlateau(), EarlyStopping()
    history, step = [], 0
    for epoch in range(epochs):
        perm = torch.from_numpy(rng.permutation(n)).to(dev)
        losses = []
        for a in range(0, n, batch_size):
            idx = perm[a:a + batch_size]
            loss = trainer.step(tm.index_select(0, idx), tv.index_select(0, idx), ts.index_select(0, idx), lr=lr,
                                dropout=dropout, seed=(seed * 1000003 + step) & 0xFFFFFFFF)
            losses.append(loss * idx.numel())
            step += 1
        train_loss = float(torch.stack(losses).sum().item()) / n
        current = trainer.model()
        val_loss = validation_loss(current, vm, vv, vs)
        history.append({"epoch": epoch, "loss": train_loss, "val_loss": val_loss, "lr": lr})
        if verbose:
            print("epoch %d: loss %.6f - val_loss %.6f - lr %.3g" % (epoch + 1, train_loss, val_loss, lr))
        if model_cache_path is not None:
            (save or (lambda m, p: m.save(p)))(current, model_cache_path)   # ModelCheckpoint
        lr = plateau.on_epoch_end(val_loss, lr)
        if stopper.on_epoch_end(val_loss):
            break
    return trainer.model(), history
