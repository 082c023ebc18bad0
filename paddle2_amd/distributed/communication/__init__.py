"""paddle.distributed.communication (reference: python/paddle/distributed/communication/): the
collective API and its ``stream`` variants, implemented in :mod:`paddle2_amd.distributed.collective`."""
from ..collective import (ReduceOp, all_gather, all_gather_object, all_reduce, alltoall, alltoall_single,  # noqa
                          barrier, batch_isend_irecv, broadcast, broadcast_object_list, gather, irecv, isend, recv,
                          reduce, reduce_scatter, scatter, scatter_object_list, send, stream)
from ..collective import P2POp  # noqa: F401
