"""Per-step communication model of group-sharded stage 3 (what one rank sends / receives over xGMI per step).

Used to size buffers and to check the first multi-GPU SCALE run against expectations (profiles/r3_stage3_comm.md).
Model of this framework's stage 3 (group_sharded.py), not the reference's (group_sharded_stage3.py:743-805 all-
reduces every parameter's full gradient and slices it; here ONE reduce-scatter per flat unit moves half of that):

  * forward: one all-gather per unit (param dtype), except the root unit (tied / shared parameters) gathered once;
  * backward: the same all-gathers again, except the last forward unit, kept gathered across the turn — or none
    at all with ``keep_gathered`` (every unit stays gathered from its forward to its backward: the MI355X default
    when the bf16 model is <= 8 % of HBM, group_sharded.GroupShardedModel._keep_gathered_policy);
  * gradients: one reduce-scatter per unit of its flat fp32 gradient (``grad_bytes`` = 4; 2 for a bf16 reduce-
    scatter, which halves the bytes but sums the ranks' partials in bf16);
  * ring algorithms: a rank moves (N-1)/N of each collective's full buffer; time = bytes / bus bandwidth.

RCCL on an 8 x MI355X node runs its rings over the point-to-point xGMI mesh (7 links per GPU); ``busbw_GBps``
is the all-gather / reduce-scatter bus bandwidth to assume (measure it with ``fleet.collective_perf`` on the
node and pass it in).
"""
from __future__ import annotations


def stage3_bytes_per_step(unit_numels, N, param_bytes=2, grad_bytes=4, root_numel=0, keep_last=True,
                          keep_gathered=False):
    """-> dict of per-rank bytes per step: ag_fwd, ag_bwd, rs, total (and the per-unit peaks)."""
    if N <= 1:
        return {"ag_fwd": 0, "ag_bwd": 0, "rs": 0, "total": 0, "max_unit_ag": 0, "max_unit_rs": 0}
    f = (N - 1) / N
    pad = [(-(-n // N)) * N for n in unit_numels]          # flat units padded to a multiple of N
    ag = [p * param_bytes * f for p in pad]
    rs = [p * grad_bytes * f for p in pad]
    root_pad = (-(-root_numel // N)) * N if root_numel else 0
    ag_fwd = sum(ag) + root_pad * param_bytes * f
    ag_bwd = 0 if keep_gathered else sum(ag) - (ag[-1] if keep_last and ag else 0)
    rs_tot = sum(rs) + root_pad * grad_bytes * f
    return {"ag_fwd": ag_fwd, "ag_bwd": ag_bwd, "rs": rs_tot, "total": ag_fwd + ag_bwd + rs_tot,
            "max_unit_ag": max(ag) if ag else 0, "max_unit_rs": max(rs) if rs else 0}


def llama_units(hidden=4096, inter=11008, layers=32, vocab=32000, heads=32, kv_heads=32):
    """Flat unit sizes of a Llama decoder stack (q/k/v/o + gate/up/down + 2 RMSNorm weights per layer) and the
    root unit (embedding, final norm, lm_head) — the units _find_units builds for models.LlamaForCausalLM."""
    hd = hidden // heads
    attn = hidden * (heads * hd) + 2 * hidden * (kv_heads * hd) + (heads * hd) * hidden
    mlp = 3 * hidden * inter
    layer = attn + mlp + 2 * hidden
    return [layer] * layers, 2 * vocab * hidden + hidden


def step_comm_time(bytes_per_step, busbw_GBps=350.0):
    """Seconds of collective time per step (not overlapped) at the given bus bandwidth."""
    return bytes_per_step / (busbw_GBps * 1e9)


def llama7b_report(N=8, busbw_GBps=350.0, grad_bytes=4, keep_gathered=True):
    units, root = llama_units()
    b = stage3_bytes_per_step(units, N, grad_bytes=grad_bytes, root_numel=root, keep_gathered=keep_gathered)
    b["seconds"] = step_comm_time(b["total"], busbw_GBps)
    return b
