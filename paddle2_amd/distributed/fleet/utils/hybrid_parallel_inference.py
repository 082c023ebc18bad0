"""Pipeline(+tensor)-parallel static inference (reference:
python/paddle/distributed/fleet/utils/hybrid_parallel_inference.py HybridParallelInferenceHelper — rank
layout :225, _insert_sendrecv_ops_for_boundaries :523, _insert_sendrecv_ops_in_while_block :660,
gen_infer_program :773).

The user records one program with ``paddle.static.device_guard("gpu:<stage>")`` annotations ("gpu:all" for
ops every stage runs, e.g. loop counters), typically a generation ``while_loop`` whose body spans the
stages.  ``gen_infer_program`` turns it, on each rank, into that rank's stage program:

* ops of other stages are dropped; a value produced on stage p and read on stage q gets a send on p right
  after its producer and a recv on q right before its first reader.  Ranks are laid out [num_pp, num_mp]
  (rank = stage * num_mp + mp_index) and a transfer goes to the same mp index of the other stage.  xGMI is
  point-to-point between every GPU pair, so a value crosses directly from p to q (the reference relays it
  through every stage in between);
* the recorded while-loop is split the same way inside its cond / body sub-programs, and because the loop
  is functional (cond(*vars) / body(*vars) -> vars) every loop-carried value produced on one stage is
  broadcast to all stages at the end of each iteration — the reference's ``sync_in_while_var_names`` /
  ``sync_in_while_lastpp2firstpp_var_names`` bookkeeping falls out of the dataflow (the names are
  accepted and checked against the loop outputs);
* transfers carry a small shape header, so dynamic batch / sequence sizes need no ``micro_batch_size`` /
  ``beam_size`` shape patching; sends are asynchronous (isend) and drained at the end of each program
  run, recvs block in program order — every rank walks the same global op order, so it cannot deadlock.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as tdist

from ....static.graph import Op, Program, VarRef

_HDR = 9   # ndim + up to 8 dims


def _world():
    if tdist.is_available() and tdist.is_initialized():
        return tdist.get_rank(), tdist.get_world_size()
    import os

    return int(os.environ.get("PADDLE_TRAINER_ID", 0)), int(os.environ.get("PADDLE_TRAINERS_NUM", 1))


def _stage_of(op):
    d = op.attrs.get("op_device") if op.attrs else None
    if not d or ":" not in d:
        return None
    tail = d.split(":")[-1]
    return None if tail == "all" else int(tail)


def _in_vids(op):
    vids = []

    def walk(x):
        if isinstance(x, VarRef):
            vids.append(x.vid)
        elif isinstance(x, (list, tuple)):
            for y in x:
                walk(y)
        elif isinstance(x, dict):
            for y in x.values():
                walk(y)

    walk(op.args)
    walk(op.kwargs)
    return vids


class _Comm:
    """Point-to-point transfers of one stage program: shape header + payload, isend kept until drained."""

    def __init__(self, helper):
        self.h = helper
        self.pending = []

    def send(self, t, dst_rank):
        hdr = torch.zeros(_HDR, dtype=torch.int64, device=t.device)
        hdr[0] = t.dim()
        if t.dim():
            hdr[1:1 + t.dim()] = torch.tensor(list(t.shape), dtype=torch.int64)
        t = t.contiguous()
        self.pending.append((tdist.isend(hdr, dst_rank), hdr))
        self.pending.append((tdist.isend(t, dst_rank), t))

    def recv(self, src_rank, dtype, device):
        hdr = torch.zeros(_HDR, dtype=torch.int64, device=device)
        tdist.recv(hdr, src_rank)
        nd = int(hdr[0])
        out = torch.empty([int(v) for v in hdr[1:1 + nd].tolist()], dtype=dtype, device=device)
        tdist.recv(out, src_rank)
        return out

    def drain(self):
        for w, _ in self.pending:
            w.wait()
        self.pending.clear()


class HybridParallelInferenceHelper:
    def __init__(self, startup_program, main_program, num_mp=1, num_pp=1, micro_batch_size=1, beam_size=1,
                 init_comm=True, role_maker=None):
        if not isinstance(main_program, Program) or not isinstance(startup_program, Program):
            raise TypeError("startup_program and main_program must be static Programs")
        self._main_program, self._startup_program = main_program, startup_program
        self.micro_batch_size, self.beam_size, self.init_comm = micro_batch_size, beam_size, init_comm
        if role_maker is not None and hasattr(role_maker, "_worker_index"):
            self.rank, self.nranks = role_maker._worker_index(), role_maker._worker_num()
        else:
            self.rank, self.nranks = _world()
        if num_mp * num_pp != self.nranks:
            raise ValueError(f"num_mp ({num_mp}) * num_pp ({num_pp}) must equal the number of ranks ({self.nranks})")
        self.num_mp, self.num_pp = num_mp, num_pp
        arr = np.arange(num_pp * num_mp).reshape(num_pp, num_mp)
        self._stage, mp_idx = divmod(self.rank, num_mp)
        self.mp_group = arr[self._stage, :].tolist()
        self.pp_group = arr[:, mp_idx].tolist()
        self._comm = _Comm(self)
        self._pipeline_pair = []   # (src stage, dst stage) pairs that exchange values (reference bookkeeping)

    # ----------------------------------------------------------------------------------------- split
    def _rank_of(self, stage):
        return self.pp_group[stage]

    def _send_op(self, vid, dst_stage):
        comm, dst = self._comm, self._rank_of(dst_stage)

        def send(t):
            comm.send(t, dst)
            return None

        send.__qualname__ = f"send_v2[to stage {dst_stage}]"
        return Op("native", send, (VarRef(vid),), {}, [], {"op_device": f"gpu:{self._stage}", "peer": dst,
                                                               "side_effect": True})

    def _recv_op(self, vid, src_stage, meta):
        comm, src = self._comm, self._rank_of(src_stage)
        dtype = meta.dtype if meta is not None else torch.float32
        helper = self

        def recv():
            return comm.recv(src, dtype, helper._device())

        recv.__qualname__ = f"recv_v2[from stage {src_stage}]"
        return Op("native", recv, (), {}, [vid], {"op_device": f"gpu:{self._stage}", "peer": src,
                                                             "side_effect": True})

    def _device(self):
        from ....framework.place import current_torch_device

        return current_torch_device()

    def _meta(self, program, vid):
        v = program.vars.get(vid)   # SymTensor: a meta-device tensor carrying the recorded dtype
        return v if isinstance(v, torch.Tensor) else None

    def _split(self, program, always_local=(), loop_outs=None):
        """Rewrite ``program.ops`` in place into this stage's ops + transfers; returns the producer-stage map."""
        from ....static.nn import _WhileRunner

        me, stages = self._stage, range(self.num_pp)
        producer, consumers = {}, {}
        for op in program.ops:
            st = _stage_of(op)
            if isinstance(op.fn, _WhileRunner):
                st = None   # the loop itself runs on every stage; its sub-programs are split below
            users = set(stages) if st is None else {st}
            for v in _in_vids(op):
                consumers.setdefault(v, set()).update(users)
            for v in op.outs:
                if v is not None:
                    producer[v] = st
        if loop_outs is not None:   # loop-carried values: every stage needs them for the next iteration
            for v in loop_outs:
                consumers.setdefault(v, set()).update(stages)
        new, have = [], set(always_local)
        for op in program.ops:
            st = _stage_of(op)
            if isinstance(op.fn, _WhileRunner):
                self._split_while(op.fn)
                st = None
            if st is not None and st != me:
                continue
            for v in _in_vids(op):
                p = producer.get(v)
                if p is not None and p != me and v not in have:
                    new.append(self._recv_op(v, p, self._meta(program, v)))
                    have.add(v)
                    if (p, me) not in self._pipeline_pair:
                        self._pipeline_pair.append((p, me))
            new.append(op)
            for v in op.outs:
                if v is None:
                    continue
                have.add(v)
                if st == me:
                    for q in sorted(consumers.get(v, ()) - {me}):
                        new.append(self._send_op(v, q))
        if loop_outs is not None:
            # loop outputs produced on another stage and never read here inside the body still arrive
            for v in loop_outs:
                p = producer.get(v)
                if p is not None and p != me and v not in have:
                    new.append(self._recv_op(v, p, self._meta(program, v)))
                    have.add(v)
        if new and (program is self._main_program or loop_outs is not None):
            comm = self._comm

            def drain():
                comm.drain()
                return None

            drain.__qualname__ = "drain_sends"
            new.append(Op("native", drain, (), {}, [], {"op_device": "gpu:all", "side_effect": True}))
        program.ops = new
        return producer

    def _split_while(self, runner):
        loop_in = set(runner.in_vids) | set(runner.free_vids)
        self._split(runner.cond_prog, always_local=loop_in)
        self._split(runner.body_prog, always_local=loop_in, loop_outs=list(runner.body_outs))

    def gen_infer_program(self, sync_in_while_lastpp2firstpp_var_names=None, sync_in_while_var_names=None,
                          debug=False):
        """Split ``main_program`` (in place) into this rank's pipeline stage; -> the stage program."""
        names = list(sync_in_while_lastpp2firstpp_var_names or []) + list(sync_in_while_var_names or [])
        if self.num_pp > 1:
            if self.init_comm and not (tdist.is_available() and tdist.is_initialized()):
                raise RuntimeError("pipeline inference needs an initialised process group (init_parallel_env)")
            known = {getattr(v, "name", None) for v in self._main_program.vars.values()}
            missing = [n for n in names if n not in known]
            if missing and debug:
                print(f"[hybrid_parallel_inference] sync vars not in the program (loop outputs are synced "
                      f"automatically): {missing}")
            self._split(self._main_program)
        if debug:
            print(f"[hybrid_parallel_inference] rank {self.rank} stage {self._stage}: "
                  f"{len(self._main_program.ops)} ops, pipeline pairs {self._pipeline_pair}")
        return self._main_program
