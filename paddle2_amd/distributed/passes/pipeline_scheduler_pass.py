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

