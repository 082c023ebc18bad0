"""Pipeline scheduler passes for static programs (reference:
python/paddle/distributed/passes/pipeline_scheduler_pass/ — pipeline_fthenb.py, pipeline_1f1b.py,
pipeline_eager_1f1b.py, pipeline_vpp.py, pipeline_zero_bubble.py; core.Job / core.Plan run by the
StandaloneExecutor with one scope per micro-batch).

A recorded training Program (forward ops, then ``backward`` / ``param_grad`` specials, then ``optimize``) is
split into typed sub-programs; a schedule turns (mode, micro-batches, stage, degree) into a job list — the
same per-stage orders as the reference passes — and ``PlanExecutor`` runs the jobs: every forward job replays
the forward sub-program for its micro-batch in its own environment (the micro-batch scope), every backward job
back-propagates that micro-batch's loss scaled by 1/num_micro_batches (gradients accumulate into the
parameters' .grad), data-parallel ranks average the accumulated gradients once, and the optimizer job steps.
"""
from __future__ import annotations

import torch

FORWARD, BACKWARD, OPT = "forward", "backward", "optimizer"
SCHEDULES = ("FThenB", "1F1B", "Eager1F1B", "VPP", "ZBH1")


class Job:
    def __init__(self, type, micro_batch_id=0):
        self._type = type
        self._micro_batch_id = int(micro_batch_id)

    def type(self):
        return self._type

    def micro_batch_id(self):
        return self._micro_batch_id

    def set_micro_batch_id(self, i):
        self._micro_batch_id = int(i)

    def __repr__(self):
        return f"{self._type}({self._micro_batch_id})"

    def __eq__(self, other):
        return isinstance(other, Job) and (self._type, self._micro_batch_id) == (other._type, other._micro_batch_id)


class Plan:
    def __init__(self, job_list, type_to_program):
        self._jobs = list(job_list)
        self._programs = dict(type_to_program)

    def job_list(self):
        return list(self._jobs)

    def job_types(self):
        return sorted(self._programs)

    def program(self, job_type):
        return self._programs[_base_type(job_type)]

    def micro_batch_num(self):
        return 1 + max((j.micro_batch_id() for j in self._jobs), default=0)


def _base_type(t):
    """forward3 / backward_b1 / backward_w -> forward / backward / backward (chunk / split suffixes)."""
    for base in (FORWARD, BACKWARD, OPT):
        if t.startswith(base):
            return base
    return t


# ------------------------------------------------------------------------------------------ job lists
def _fthenb(m):
    return [Job(FORWARD, i) for i in range(m)] + [Job(BACKWARD, i) for i in range(m)] + [Job(OPT, 0)]


def _one_f_one_b(m, stage, degree, eager=False):
    warm = 2 * (degree - stage) - 1 if eager else degree - stage
    if warm > m:
        raise ValueError(f"num_micro_batches ({m}) must cover the {'eager ' if eager else ''}1F1B warmup ({warm})")
    jobs, f, b = [], 0, 0
    for _ in range(warm):
        jobs.append(Job(FORWARD, f))
        f += 1
    for _ in range(m - warm):
        jobs += [Job(BACKWARD, b), Job(FORWARD, f)]
        b += 1
        f += 1
    for _ in range(warm):
        jobs.append(Job(BACKWARD, b))
        b += 1
    return jobs + [Job(OPT, 0)]


def _vpp(m, stage, degree, chunks, split_backward=False):
    if m % degree:
        raise ValueError("VPP needs num_micro_batches divisible by the pipeline degree")
    fwd_cnt, bwd_cnt = [0] * chunks, [0] * chunks

    def chunk_of(step, forward):
        c = (step % (degree * chunks)) // degree
        return c if forward else chunks - c - 1

    total = m * chunks
    if m == degree:
        warm = total
    else:
        warm = min((degree - stage - 1) * 2 + (chunks - 1) * degree, total)
    split = split_backward and m == degree
    bname = BACKWARD + ("_b" if split else "")
    jobs = []

    def fwd(step):
        c = chunk_of(step, True)
        jobs.append(Job(FORWARD + str(c), fwd_cnt[c]))
        fwd_cnt[c] += 1

    def bwd(step):
        c = chunk_of(step, False)
        jobs.append(Job(bname + str(c), bwd_cnt[c]))
        bwd_cnt[c] += 1

    for s in range(warm):
        fwd(s)
    for s in range(total - warm):
        fwd(s + warm)
        bwd(s)
    for s in range(total - warm, total):
        bwd(s)
    if split:
        for c in range(chunks):
            for i in range(m):
                jobs.append(Job(BACKWARD + "_w" + str(c), i))
    return jobs + [Job(OPT, 0)]


def _zbh1(m, stage, degree):
    if degree > m:
        raise ValueError("ZBH1 needs num_micro_batches >= the pipeline degree")
    warm = degree - stage
    jobs, f, b = [], 0, 0
    for _ in range(warm):
        jobs.append(Job(FORWARD, f))
        f += 1
    for _ in range(stage):
        jobs += [Job(BACKWARD + "_b", b), Job(FORWARD, f)]
        b += 1
        f += 1
    for _ in range(m - degree):
        jobs += [Job(BACKWARD, b), Job(FORWARD, f)]
        f += 1
        b += 1
    for _ in range(warm - 1):
        jobs.append(Job(BACKWARD, b))
        b += 1
    if stage > 0:
        jobs += [Job(BACKWARD + "_b", b), Job(BACKWARD + "_w", b)]
    else:
        jobs.append(Job(BACKWARD, b))
    for i in range(stage):
        jobs.append(Job(BACKWARD + "_w", i))
    return jobs + [Job(OPT, 0)]


def create_job_list(schedule_mode, num_micro_batches, pp_stage=0, pp_degree=1, vpp_degree=1, split_backward=False):
    if schedule_mode == "FThenB":
        return _fthenb(num_micro_batches)
    if schedule_mode == "1F1B":
        return _one_f_one_b(num_micro_batches, pp_stage, pp_degree)
    if schedule_mode == "Eager1F1B":
        return _one_f_one_b(num_micro_batches, pp_stage, pp_degree, eager=True)
    if schedule_mode == "VPP":
        return _vpp(num_micro_batches, pp_stage, pp_degree, vpp_degree, split_backward)
    if schedule_mode == "ZBH1":
        return _zbh1(num_micro_batches, pp_stage, pp_degree)
    raise ValueError(f"unknown schedule_mode {schedule_mode!r}; one of {SCHEDULES}")


# ------------------------------------------------------------------------------------------ program split
def split_program(program):
    """Recorded training Program -> {forward, backward, optimizer} sub-programs (op-role split)."""
    from ...static.graph import Program

    parts = {FORWARD: Program(), BACKWARD: Program(), OPT: Program()}
    for p in parts.values():
        p.feeds, p.vars = program.feeds, program.vars
    for op in program.ops:
        if op.kind in ("backward", "grad", "param_grad"):
            parts[BACKWARD].ops.append(op)
        elif op.kind == "optimize":
            parts[OPT].ops.append(op)
        else:
            parts[FORWARD].ops.append(op)
    return parts


def apply_pass(program, schedule_mode="1F1B", num_micro_batches=1, pp_stage=0, pp_degree=1, vpp_degree=1,
               split_backward=False):
    """-> Plan (the reference's ``apply_pass(main, startup, ctx)`` result)."""
    return Plan(create_job_list(schedule_mode, num_micro_batches, pp_stage, pp_degree, vpp_degree, split_backward),
                split_program(program))


# ------------------------------------------------------------------------------------------ execution
class PlanExecutor:
    """Runs a Plan over per-micro-batch feeds (one environment = the micro-batch scope per micro-batch)."""

    def __init__(self, executor=None, dp_group=None):
        from ...static import Executor

        self._exe = executor or Executor()
        self._dp_group = dp_group

    def run(self, program, plan, micro_feeds, fetch_list=()):
        from ...static.executor import _feed_tensor

        m = len(micro_feeds)
        fwd = plan.program(FORWARD)
        bwd = plan.program(BACKWARD)
        loss_vid = next((op.attrs["loss"] for op in bwd.ops if op.kind == "backward"), None)
        fetch_ids = [self._exe._fetch_id(program, f) for f in fetch_list]
        envs = [None] * m
        fetched = [None] * m
        optimizers = [op.attrs["optimizer"] for op in plan.program(OPT).ops]
        backed = set()
        for job in plan.job_list():
            t, i = _base_type(job.type()), job.micro_batch_id()
            if t == FORWARD:
                env = {}
                for name, v in micro_feeds[i].items():
                    sym = program.feeds[name]
                    env[sym._vid] = _feed_tensor(v, sym, self._exe._device)
                with torch.enable_grad():
                    envs[i] = self._exe._replay(fwd, env, grad=True)
                fetched[i] = [envs[i][f] for f in fetch_ids]
            elif t == BACKWARD:
                if job.type().startswith(BACKWARD + "_w") or i in backed:
                    continue   # weight-grad half: produced together with the input grad by autograd
                backed.add(i)
                if loss_vid is not None:
                    (envs[i][loss_vid] / m).backward()
                for op in bwd.ops:
                    if op.kind == "param_grad":
                        g = op.attrs["param"]._t.grad
                        envs[i][op.attrs["out"]] = g if g is not None else torch.zeros_like(op.attrs["param"]._t)
                envs[i] = {k: v for k, v in envs[i].items() if k in fetch_ids}   # free activations
            elif t == OPT:
                self._average_grads(optimizers)
                with torch.no_grad():
                    for opt in optimizers:
                        opt.step()
                        opt.clear_grad(set_to_zero=False)
        return fetched

    def _average_grads(self, optimizers):
        """Data parallelism: one all-reduce (average) of the accumulated gradients per step."""
        import torch.distributed as tdist

        if not tdist.is_initialized() or tdist.get_world_size() == 1:
            return
        from ..collective import ReduceOp, all_reduce
        from ...framework.tensor import Tensor

        for opt in optimizers:
            for p in opt._parameter_list:
                g = p._t.grad
                if g is None:
                    continue
                all_reduce(Tensor._wrap(g), op=ReduceOp.AVG if tdist.get_backend() != "gloo" else ReduceOp.SUM,
                           group=self._dp_group)
                if tdist.get_backend() == "gloo":
                    g.div_(tdist.get_world_size())



# ------------------------------------------------------------------------------------------ stage execution
def _op_stage(op):
    """-> pipeline stage of a recorded op from its ``op_device`` ("gpu:<k>"), "all" for "gpu:all", None when
    unannotated."""
    d = op.attrs.get("op_device") if op.attrs else None
    if not d or ":" not in d:
        return None
    tail = d.split(":")[-1]
    return "all" if tail == "all" else int(tail)


class StagePlanExecutor:
    """Runs a Plan on ONE stage of a pipeline group: the multi-rank form of ``PlanExecutor`` (reference: the
    pipeline passes give each pp rank the ops of its stage plus send_v2 / recv_v2 at the stage boundaries, and the
    StandaloneExecutor runs that rank's job list; python/paddle/distributed/passes/pipeline_scheduler_pass/
    pipeline_pass_base.py, pass_utils.py ``_split_program_into_forward_backward_optimize``).

    The forward program's ops are assigned to stages by their ``paddle.static.device_guard("gpu:<k>")`` annotation
    (unannotated ops stay on the stage of the op before them; "gpu:all" ops run on every stage).  A value produced
    on stage p and read on stage q crosses p -> q directly (xGMI links every GPU pair) with a shape header, so
    micro-batches of any size need no shape patching.  Per job of this stage's list:

    * forward(i): receive the micro-batch's boundary inputs (as leaves that require grad), replay this stage's ops
      with autograd on, send the boundary outputs (isend, drained at the end of the step);
    * backward(i): on the loss stage back-propagate loss_i / num_micro_batches, elsewhere receive the gradients of
      the sent outputs (summed over consumers) and back-propagate them; then send the received inputs' gradients
      back to their producers — parameter gradients accumulate in ``.grad`` over the micro-batches;
    * optimizer: average the accumulated gradients over ``dp_group`` (if any) and step — parameters of other
      stages have no gradient and are skipped by the optimizer.

    Receives block in job order and sends are asynchronous; every schedule of ``create_job_list`` orders each
    stage's jobs so that a receive only waits on jobs its peer has already issued, hence no deadlock.
    """

    def __init__(self, program, plan, pp_ranks=None, executor=None, dp_group=None):
        import torch.distributed as tdist

        from ...static import Executor
        from ...static.graph import Program
        from ..fleet.utils.hybrid_parallel_inference import _Comm, _in_vids

        self._exe = executor or Executor()
        self._dp_group = dp_group
        rank = tdist.get_rank() if tdist.is_initialized() else 0
        self.pp_ranks = list(pp_ranks) if pp_ranks is not None else list(
            range(tdist.get_world_size() if tdist.is_initialized() else 1))
        if rank not in self.pp_ranks:
            raise ValueError(f"rank {rank} is not in the pipeline group {self.pp_ranks}")
        self.stage = self.pp_ranks.index(rank)
        self.program, self.plan = program, plan
        fwd = plan.program(FORWARD)
        stages, cur = [], 0
        for op in fwd.ops:
            s = _op_stage(op)
            if s is None:
                s = cur
            elif s != "all":
                if s >= len(self.pp_ranks):
                    raise ValueError(f"op placed on stage {s} but the pipeline has {len(self.pp_ranks)} stages")
                cur = s
            stages.append(s)
        producer, pidx, consumers = {}, {}, {}
        for i, (op, s) in enumerate(zip(fwd.ops, stages)):
            for v in _in_vids(op):
                consumers.setdefault(v, set()).update(range(len(self.pp_ranks)) if s == "all" else {s})
            for v in op.outs:
                if v is not None:
                    producer[v], pidx[v] = s, i
        me = self.stage
        local = Program()
        local.feeds, local.vars = fwd.feeds, fwd.vars
        local.ops = [op for op, s in zip(fwd.ops, stages) if s == me or s == "all"]
        self._local = local
        reads = {v for op in local.ops for v in _in_vids(op)}
        # boundary values in producer-op order on both sides of every pair (the message order of a channel)
        self._recv = sorted(((v, producer[v]) for v in reads if producer.get(v) not in (None, me, "all")),
                            key=lambda e: pidx[e[0]])
        self._send = sorted(((v, sorted(consumers.get(v, set()) - {me})) for v, s in producer.items()
                             if s == me and consumers.get(v, set()) - {me}), key=lambda e: pidx[e[0]])
        bwd = plan.program(BACKWARD)
        self._loss = next((op.attrs["loss"] for op in bwd.ops if op.kind == "backward"), None)
        self._loss_local = self._loss is not None and producer.get(self._loss) in (me, "all")
        self._comm = _Comm(None)
        self._optimizers = [op.attrs["optimizer"] for op in plan.program(OPT).ops]

    def _dtype(self, vid):
        v = self.program.vars.get(vid)
        return v.dtype if isinstance(v, torch.Tensor) else torch.float32

    def run(self, micro_feeds, fetch_list=()):
        """-> per micro-batch list of the fetch values this stage holds (None for values of other stages)."""
        from ...static.executor import _feed_tensor

        exe, m = self._exe, len(micro_feeds)
        dev = exe._device
        fetch_ids = [exe._fetch_id(self.program, f) for f in fetch_list]
        envs, recvd, fetched = [None] * m, [None] * m, [None] * m
        rank_of = self.pp_ranks.__getitem__
        for job in self.plan.job_list():
            t, i = _base_type(job.type()), job.micro_batch_id()
            if t == FORWARD:
                env, got = {}, {}
                for name, v in micro_feeds[i].items():
                    sym = self.program.feeds[name]
                    env[sym._vid] = _feed_tensor(v, sym, dev)
                for vid, src in self._recv:
                    x = self._comm.recv(rank_of(src), self._dtype(vid), dev)
                    if x.is_floating_point():
                        x.requires_grad_(True)
                    env[vid] = got[vid] = x
                with torch.enable_grad():
                    envs[i] = exe._replay(self._local, env, grad=True)
                recvd[i] = got
                for vid, dsts in self._send:
                    for q in dsts:
                        self._comm.send(envs[i][vid].detach(), rank_of(q))
                fetched[i] = [envs[i].get(f) for f in fetch_ids]
            elif t == BACKWARD:
                if job.type().startswith(BACKWARD + "_w"):
                    continue   # weight-grad half: autograd produces it together with the input gradient
                env = envs[i]
                outs, grads = [], []
                if self._loss_local:
                    outs.append(env[self._loss] / m)
                    grads.append(None)
                for vid, dsts in self._send:
                    gsum = None
                    for q in dsts:
                        if not self._dtype(vid).is_floating_point:
                            continue
                        g = self._comm.recv(rank_of(q), self._dtype(vid), dev)
                        gsum = g if gsum is None else gsum + g
                    x = env[vid]
                    if gsum is not None and isinstance(x, torch.Tensor) and x.requires_grad:
                        outs.append(x)
                        grads.append(gsum)
                if outs:
                    torch.autograd.backward(outs, [g if g is not None else torch.ones_like(o)
                                                   for o, g in zip(outs, grads)])
                for vid, src in self._recv:
                    x = recvd[i][vid]
                    if not x.is_floating_point():
                        continue
                    g = x.grad if x.grad is not None else torch.zeros_like(x)
                    self._comm.send(g, rank_of(src))
                envs[i] = {k: v for k, v in env.items() if k in fetch_ids}   # free the activations
                recvd[i] = None
            elif t == OPT:
                self._comm.drain()
                self._average_grads()
                with torch.no_grad():
                    for opt in self._optimizers:
                        opt.step()
                        opt.clear_grad(set_to_zero=False)
        self._comm.drain()
        return fetched

    def _average_grads(self):
        import torch.distributed as tdist

        if self._dp_group is None or not tdist.is_initialized():
            return
        n = tdist.get_world_size(self._dp_group)
        if n == 1:
            return
        for opt in self._optimizers:
            for p in opt._parameter_list:
                g = p._t.grad
                if g is not None:
                    tdist.all_reduce(g, group=self._dp_group)
                    g.div_(n)
