"""paddle.incubate.multiprocessing (reference: python/paddle/incubate/multiprocessing/{__init__,reductions}.py):
the standard ``multiprocessing`` API with framework Tensors shareable between processes.  ``init_reductions``
registers a reducer so a Tensor sent through a multiprocessing Queue / Pipe is rebuilt on the other side over the
same storage — CPU tensors through shared memory, device tensors through the IPC handles of torch's reductions
(HIP IPC memory handles; dmabuf IPC on this pool, HSA_ENABLE_IPC_MODE_LEGACY=0)."""
from multiprocessing import *  # noqa: F401,F403
from multiprocessing.reduction import ForkingPickler

__all__ = ["init_reductions"]


def _rebuild_tensor(raw, stop_gradient, name):
    from ...framework.tensor import Tensor

    t = Tensor._wrap(raw)
    t.stop_gradient = stop_gradient
    if name is not None:
        try:
            t.name = name
        except AttributeError:
            pass
    return t


def _reduce_tensor(t):
    raw = t._t.detach()
    if not raw.is_cuda:
        raw = raw.share_memory_()
    return _rebuild_tensor, (raw, bool(t.stop_gradient), getattr(t, "name", None))


def init_reductions():
    import torch.multiprocessing  # noqa: F401  (registers torch.Tensor's shared-memory / IPC reducers)

    from ...framework.tensor import Tensor

    ForkingPickler.register(Tensor, _reduce_tensor)
    for sub in Tensor.__subclasses__():
        ForkingPickler.register(sub, _reduce_tensor)


init_reductions()
