"""High-level API: ``paddle.Model`` (reference: python/paddle/hapi/model.py:1472, fit :2200,
DynamicGraphAdapter :1196, train_batch :1237) and callbacks (hapi/callbacks.py)."""
from __future__ import annotations

import os
import time

import numpy as np
import torch

from ..framework.tensor import Tensor
from ..io import DataLoader, Dataset, DistributedBatchSampler
from ..metric import Metric
from . import callbacks as cbks
from .callbacks import Callback  # noqa: F401


def _to_list(x):
    if x is None:
        return []
    return list(x) if isinstance(x, (list, tuple)) else [x]


def _as_tensor(x):
    if isinstance(x, Tensor):
        return x
    from ..framework.tensor import to_tensor

    return to_tensor(np.asarray(x))


class Model:
    def __init__(self, network, inputs=None, labels=None):
        self.network = network
        self._inputs = inputs
        self._labels = labels
        self._optimizer = None
        self._loss = None
        self._metrics = []
        self._amp_level = "O0"
        self._scaler = None
        self.stop_training = False

    # ------------------------------------------------------------ setup
    def prepare(self, optimizer=None, loss=None, metrics=None, amp_configs=None):
        self._optimizer = optimizer
        self._loss = loss
        self._metrics = _to_list(metrics)
        for m in self._metrics:
            assert isinstance(m, Metric), "metrics must be paddle.metric.Metric instances"
        if amp_configs is not None:
            cfg = {"level": amp_configs} if isinstance(amp_configs, str) else dict(amp_configs)
            self._amp_level = cfg.get("level", "O1")
            self._amp_dtype = cfg.get("dtype", "bfloat16")
            if self._amp_level == "O2":
                from .. import amp

                amp.decorate(self.network, optimizer, level="O2", dtype=self._amp_dtype)
            if self._amp_dtype == "float16":
                from ..amp import GradScaler

                self._scaler = GradScaler(init_loss_scaling=cfg.get("init_loss_scaling", 2.0 ** 15))

    def parameters(self, *args, **kwargs):
        return self.network.parameters(*args, **kwargs)

    # ------------------------------------------------------------ batch steps
    def _forward(self, inputs):
        if self._amp_level in ("O1", "O2"):
            from ..amp import auto_cast

            with auto_cast(level=self._amp_level, dtype=self._amp_dtype):
                return self.network(*inputs)
        return self.network(*inputs)

    def train_batch(self, inputs, labels=None, update=True):
        self.network.train()
        inputs = [_as_tensor(x) for x in _to_list(inputs)]
        labels = [_as_tensor(x) for x in _to_list(labels)]
        outputs = self._forward(inputs)
        outs = _to_list(outputs)
        losses = self._loss(*(outs + labels))
        losses = _to_list(losses)
        final = losses[0] if len(losses) == 1 else sum(losses[1:], losses[0])
        if self._scaler is not None:
            self._scaler.scale(final).backward()
        else:
            final.backward()
        if update:
            if self._scaler is not None:
                self._scaler.step(self._optimizer)
                self._scaler.update()
            else:
                self._optimizer.step()
            self._optimizer.clear_grad()
        metrics = []
        for m in self._metrics:
            r = m.compute(*(outs + labels))
            metrics.append(m.update(*[x for x in _to_list(r)]))
        loss_np = [float(l.item()) for l in losses]
        return (loss_np, metrics) if metrics else loss_np

    @torch.no_grad()
    def eval_batch(self, inputs, labels=None):
        self.network.eval()
        inputs = [_as_tensor(x) for x in _to_list(inputs)]
        labels = [_as_tensor(x) for x in _to_list(labels)]
        outs = _to_list(self._forward(inputs))
        metrics = []
        losses = []
        if self._loss is not None and labels:
            losses = [float(l.item()) for l in _to_list(self._loss(*(outs + labels)))]
        for m in self._metrics:
            r = m.compute(*(outs + labels))
            metrics.append(m.update(*[x for x in _to_list(r)]))
        return (losses, metrics) if metrics else losses

    @torch.no_grad()
    def predict_batch(self, inputs):
        self.network.eval()
        inputs = [_as_tensor(x) for x in _to_list(inputs)]
        outs = _to_list(self._forward(inputs))
        return [o.numpy() for o in outs]

    # ------------------------------------------------------------ loops
    def _loader(self, data, batch_size, shuffle, drop_last, num_workers):
        if data is None or isinstance(data, DataLoader):
            return data
        if isinstance(data, Dataset):
            from ..distributed import collective as C

            if C.get_world_size() > 1:
                bs = DistributedBatchSampler(data, batch_size, shuffle=shuffle, drop_last=drop_last)
                return DataLoader(data, batch_sampler=bs, num_workers=num_workers)
            return DataLoader(data, batch_size=batch_size, shuffle=shuffle, drop_last=drop_last,
                              num_workers=num_workers)
        return data

    def _split(self, batch):
        batch = _to_list(batch)
        n_in = len(self._inputs) if self._inputs is not None else max(1, len(batch) - 1)
        return batch[:n_in], batch[n_in:]

    def fit(self, train_data=None, eval_data=None, batch_size=1, epochs=1, eval_freq=1, log_freq=10, save_dir=None,
            save_freq=1, verbose=2, drop_last=False, shuffle=True, num_workers=0, callbacks=None,
            accumulate_grad_batches=1, num_iters=None):
        loader = self._loader(train_data, batch_size, shuffle, drop_last, num_workers)
        eval_loader = self._loader(eval_data, batch_size, False, False, num_workers)
        cb = cbks.config_callbacks(callbacks, model=self, epochs=epochs,
                                   steps=len(loader) if hasattr(loader, "__len__") else None, log_freq=log_freq,
                                   save_freq=save_freq, save_dir=save_dir, verbose=verbose,
                                   metrics=self._metrics_name())
        self.stop_training = False
        cb.on_train_begin()
        it = 0
        history = []
        for epoch in range(epochs):
            cb.on_epoch_begin(epoch)
            for m in self._metrics:
                m.reset()
            logs = {}
            for step, batch in enumerate(loader):
                cb.on_train_batch_begin(step)
                ins, labs = self._split(batch)
                update = (step + 1) % accumulate_grad_batches == 0
                res = self.train_batch(ins, labs, update=update)
                logs = self._logs(res)
                logs["step"] = step
                logs["batch_size"] = batch_size
                cb.on_train_batch_end(step, logs)
                it += 1
                if num_iters is not None and it >= num_iters:
                    self.stop_training = True
                    break
            history.append(logs)
            if eval_loader is not None and (epoch + 1) % eval_freq == 0:
                self.evaluate(eval_loader, batch_size, log_freq, verbose=0)
            cb.on_epoch_end(epoch, logs)
            if self.stop_training:
                break
        cb.on_train_end(logs)
        return history

    def _metrics_name(self):
        names = ["loss"]
        for m in self._metrics:
            n = m.name()
            names.extend(n if isinstance(n, list) else [n])
        return names

    def _logs(self, res):
        logs = {}
        if isinstance(res, tuple):
            loss, metrics = res
        else:
            loss, metrics = res, []
        logs["loss"] = loss
        for m in self._metrics:
            acc = m.accumulate()
            n = m.name()
            if isinstance(n, list):
                if isinstance(acc, list):
                    for k, v in zip(n, acc):
                        logs[k] = v
                else:
                    logs[n[0]] = acc
            else:
                logs[n] = acc
        return logs

    def evaluate(self, eval_data, batch_size=1, log_freq=10, verbose=2, num_workers=0, callbacks=None,
                 num_iters=None):
        loader = self._loader(eval_data, batch_size, False, False, num_workers)
        for m in self._metrics:
            m.reset()
        losses = []
        for i, batch in enumerate(loader):
            ins, labs = self._split(batch)
            r = self.eval_batch(ins, labs)
            l = r[0] if isinstance(r, tuple) else r
            if l:
                losses.append(l[0])
            if num_iters is not None and i + 1 >= num_iters:
                break
        out = {"loss": [float(np.mean(losses))] if losses else []}
        for m in self._metrics:
            n = m.name()
            acc = m.accumulate()
            if isinstance(n, list):
                if isinstance(acc, list):
                    out.update(dict(zip(n, acc)))
                else:
                    out[n[0]] = acc
            else:
                out[n] = acc
        if verbose:
            print("Eval samples:", out)
        return out

    def predict(self, test_data, batch_size=1, num_workers=0, stack_outputs=False, verbose=1, callbacks=None):
        loader = self._loader(test_data, batch_size, False, False, num_workers)
        outs = []
        for batch in loader:
            ins, _ = self._split(batch)
            if self._inputs is None:
                ins = _to_list(batch)[:1]
            outs.append(self.predict_batch(ins))
        res = list(zip(*outs))
        if stack_outputs:
            res = [np.concatenate(r, 0) for r in res]
        return res

    # ------------------------------------------------------------ persistence
    def save(self, path, training=True):
        from ..framework.io import save

        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        save(self.network.state_dict(), path + ".pdparams")
        if training and self._optimizer is not None:
            save(self._optimizer.state_dict(), path + ".pdopt")

    def load(self, path, skip_mismatch=False, reset_optimizer=False):
        from ..framework.io import load

        sd = load(path + ".pdparams" if not path.endswith(".pdparams") else path)
        self.network.set_state_dict(sd)
        opt_path = (path[:-9] if path.endswith(".pdparams") else path) + ".pdopt"
        if not reset_optimizer and self._optimizer is not None and os.path.exists(opt_path):
            self._optimizer.set_state_dict(load(opt_path))

    def summary(self, input_size=None, dtype=None):
        return summary(self.network, input_size, dtypes=dtype)


def summary(net, input_size=None, dtypes=None, input=None):
    total = sum(p.size for p in net.parameters())
    trainable = sum(p.size for p in net.parameters() if not p.stop_gradient)
    print(f"Total params: {total:,}\nTrainable params: {trainable:,}\nNon-trainable params: {total - trainable:,}")
    return {"total_params": total, "trainable_params": trainable}


def flops(net, input_size, custom_ops=None, print_detail=False):
    """Count multiply-accumulate FLOPs of Linear/Conv layers with forward hooks."""
    from ..nn import Conv2D, Linear
    from ..tensor.random import rand

    total = [0]

    def hook(layer, inp, out):
        if isinstance(layer, Linear):
            total[0] += int(np.prod(out.shape)) * layer.weight.shape[0]
        elif isinstance(layer, Conv2D):
            k = int(np.prod(layer.weight.shape[1:]))
            total[0] += int(np.prod(out.shape)) * k

    hs = [l.register_forward_post_hook(hook) for l in net.sublayers() if isinstance(l, (Linear, Conv2D))]
    with torch.no_grad():
        net(rand(input_size))
    for h in hs:
        h.remove()
    if print_detail:
        print(f"Total Flops: {total[0]}")
    return total[0]
