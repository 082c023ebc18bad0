"""hapi callbacks (reference: python/paddle/hapi/callbacks.py)."""
from __future__ import annotations

import numbers
import os
import time


class Callback:
    def __init__(self):
        self.model = None
        self.params = {}

    def set_params(self, params):
        self.params = params

    def set_model(self, model):
        self.model = model

    def on_train_begin(self, logs=None): ...
    def on_train_end(self, logs=None): ...
    def on_eval_begin(self, logs=None): ...
    def on_eval_end(self, logs=None): ...
    def on_predict_begin(self, logs=None): ...
    def on_predict_end(self, logs=None): ...
    def on_epoch_begin(self, epoch, logs=None): ...
    def on_epoch_end(self, epoch, logs=None): ...
    def on_train_batch_begin(self, step, logs=None): ...
    def on_train_batch_end(self, step, logs=None): ...
    def on_eval_batch_begin(self, step, logs=None): ...
    def on_eval_batch_end(self, step, logs=None): ...
    def on_predict_batch_begin(self, step, logs=None): ...
    def on_predict_batch_end(self, step, logs=None): ...


class CallbackList:
    def __init__(self, callbacks):
        self.callbacks = callbacks

    def __getattr__(self, name):
        def call(*a, **k):
            for c in self.callbacks:
                getattr(c, name)(*a, **k)

        return call


class ProgBarLogger(Callback):
    def __init__(self, log_freq=1, verbose=2):
        super().__init__()
        self.log_freq, self.verbose = log_freq, verbose

    def on_epoch_begin(self, epoch, logs=None):
        self.epoch = epoch
        self.t0 = time.time()
        if self.verbose:
            print(f"Epoch {epoch + 1}/{self.params.get('epochs', '?')}")

    def on_train_batch_end(self, step, logs=None):
        if self.verbose and step % self.log_freq == 0:
            items = []
            for k, v in (logs or {}).items():
                if k in ("step", "batch_size"):
                    continue
                if isinstance(v, list):
                    v = v[0] if len(v) == 1 else v
                items.append(f"{k}: {v:.4f}" if isinstance(v, numbers.Number) else f"{k}: {v}")
            print(f"step {step + 1}/{self.params.get('steps', '?')} - " + " - ".join(items), flush=True)


class ModelCheckpoint(Callback):
    def __init__(self, save_freq=1, save_dir=None):
        super().__init__()
        self.save_freq, self.save_dir = save_freq, save_dir

    def on_epoch_end(self, epoch, logs=None):
        if self.save_dir and (epoch + 1) % self.save_freq == 0:
            self.model.save(os.path.join(self.save_dir, str(epoch)))

    def on_train_end(self, logs=None):
        if self.save_dir:
            self.model.save(os.path.join(self.save_dir, "final"))


class EarlyStopping(Callback):
    def __init__(self, monitor="loss", mode="auto", patience=0, verbose=1, min_delta=0, baseline=None,
                 save_best_model=True):
        super().__init__()
        self.monitor, self.patience, self.min_delta = monitor, patience, abs(min_delta)
        self.mode = mode if mode != "auto" else ("max" if "acc" in monitor else "min")
        self.best = baseline
        self.wait = 0

    def on_epoch_end(self, epoch, logs=None):
        v = (logs or {}).get(self.monitor)
        if v is None:
            return
        v = v[0] if isinstance(v, list) else v
        better = self.best is None or (v < self.best - self.min_delta if self.mode == "min" else v > self.best + self.min_delta)
        if better:
            self.best, self.wait = v, 0
        else:
            self.wait += 1
            if self.wait > self.patience:
                self.model.stop_training = True


class LRScheduler(Callback):
    def __init__(self, by_step=True, by_epoch=False):
        super().__init__()
        self.by_step, self.by_epoch = by_step, by_epoch

    def _step(self):
        from ..optimizer.lr import LRScheduler as S

        opt = self.model._optimizer
        if opt is not None and isinstance(opt._learning_rate, S):
            opt._learning_rate.step()

    def on_train_batch_end(self, step, logs=None):
        if self.by_step:
            self._step()

    def on_epoch_end(self, epoch, logs=None):
        if self.by_epoch:
            self._step()


class VisualDL(Callback):
    def __init__(self, log_dir):
        super().__init__()
        self.log_dir = log_dir


class WandbCallback(Callback):
    pass


class ReduceLROnPlateau(Callback):
    def __init__(self, monitor="loss", factor=0.1, patience=10, verbose=1, mode="auto", min_delta=1e-4, cooldown=0,
                 min_lr=0):
        super().__init__()
        self.monitor, self.factor, self.patience, self.min_lr = monitor, factor, patience, min_lr
        self.best, self.wait = None, 0

    def on_epoch_end(self, epoch, logs=None):
        v = (logs or {}).get(self.monitor)
        if v is None:
            return
        v = v[0] if isinstance(v, list) else v
        if self.best is None or v < self.best:
            self.best, self.wait = v, 0
        else:
            self.wait += 1
            if self.wait > self.patience:
                opt = self.model._optimizer
                if not hasattr(opt._learning_rate, "step"):
                    opt.set_lr(max(opt.get_lr() * self.factor, self.min_lr))
                self.wait = 0


def config_callbacks(callbacks=None, model=None, batch_size=None, epochs=None, steps=None, log_freq=2, verbose=2,
                     save_freq=1, save_dir=None, metrics=None, mode="train"):
    cbs = list(callbacks or [])
    if not any(isinstance(c, ProgBarLogger) for c in cbs) and verbose:
        cbs.insert(0, ProgBarLogger(log_freq, verbose))
    if not any(isinstance(c, ModelCheckpoint) for c in cbs):
        cbs.append(ModelCheckpoint(save_freq, save_dir))
    for c in cbs:
        c.set_model(model)
        c.set_params({"epochs": epochs, "steps": steps, "verbose": verbose, "metrics": metrics})
    return CallbackList(cbs)
