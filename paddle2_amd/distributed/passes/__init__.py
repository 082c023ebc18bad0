"""Distributed program passes (reference: python/paddle/distributed/passes/): pipeline scheduler passes
(FThenB / 1F1B / Eager1F1B / VPP / ZBH1) producing job plans for static programs."""
from .pipeline_scheduler_pass import (BACKWARD, FORWARD, OPT, Job, Plan, PlanExecutor, StagePlanExecutor,  # noqa: F401
                                      apply_pass, create_job_list, split_program)


def new_pass(name, attrs=None):
    """Reference-style factory: new_pass("pipeline_scheduler_1F1B", {...}).apply(program) -> Plan."""
    mode = name.replace("pipeline_scheduler_", "")
    attrs = dict(attrs or {})

    class _Pass:
        def apply(self, program):
            return apply_pass(program, mode, attrs.get("num_micro_batches", 1), attrs.get("pp_stage", 0),
                              attrs.get("pp_degree", 1), attrs.get("vpp_degree", 1),
                              attrs.get("split_backward", False))

    return _Pass()
