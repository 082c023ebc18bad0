"""Sequence decoding: Decoder, BeamSearchDecoder, dynamic_decode and gather_tree
(reference: python/paddle/nn/decode.py — Decoder :62, BeamSearchDecoder :133, _beam_search_step :498,
_dynamic_decode_imperative :695; phi gather_tree kernel).

Beam search keeps every beam of every batch row in one merged ``[B * beam, ...]`` batch so the cell runs
as one batched call per step (one GEMM-shaped launch set on the GPU instead of B*beam small ones); the
per-step top-k is over the flattened ``beam * vocab`` scores.  The only host sync per step is the
"all finished" test that ends the loop, as in the reference's dygraph loop.
"""
from __future__ import annotations

from typing import NamedTuple

import torch

from ..framework.tensor import Tensor

_wrap = Tensor._wrap


def _t(x):
    return x._t if isinstance(x, Tensor) else x


def _map(fn, *structs):
    s0 = structs[0]
    if isinstance(s0, tuple) and hasattr(s0, "_fields"):
        return type(s0)(*(_map(fn, *parts) for parts in zip(*structs)))
    if isinstance(s0, (tuple, list)):
        return type(s0)(_map(fn, *parts) for parts in zip(*structs))
    if s0 is None:
        return None
    return fn(*structs)


def gather_tree(ids, parents):
    """Back-trace beam-search ids ``[T, B, beam]`` through ``parents`` (same shape) into full sequences."""
    i, p = _t(ids), _t(parents)
    T = i.shape[0]
    out = torch.empty_like(i)
    out[T - 1] = i[T - 1]
    parent = p[T - 1]
    for s in range(T - 2, -1, -1):
        out[s] = i[s].gather(-1, parent)
        parent = p[s].gather(-1, parent)
    return _wrap(out)


class Decoder:
    """Interface of a step-wise decoder driven by ``dynamic_decode``."""

    def initialize(self, inits):
        raise NotImplementedError

    def step(self, time, inputs, states, **kwargs):
        raise NotImplementedError

    def finalize(self, outputs, final_states, sequence_lengths):
        raise NotImplementedError

    @property
    def tracks_own_finished(self):
        return False


class BeamSearchDecoder(Decoder):
    """Beam search over an RNN cell: ``cell(inputs, states) -> (outputs, new_states)``; ``embedding_fn``
    maps token ids to the next inputs, ``output_fn`` maps cell outputs to vocabulary logits."""

    class OutputWrapper(NamedTuple):
        scores: object
        predicted_ids: object
        parent_ids: object

    class StateWrapper(NamedTuple):
        cell_states: object
        log_probs: object
        finished: object
        lengths: object

    kinf = 1e9

    def __init__(self, cell, start_token, end_token, beam_size, embedding_fn=None, output_fn=None):
        self.cell = cell
        self.start_token = int(start_token)
        self.end_token = int(end_token)
        self.beam_size = int(beam_size)
        self.embedding_fn = embedding_fn
        self.output_fn = output_fn
        self.batch_size = None

    # --------------------------------------------------------------------------- layout helpers
    @staticmethod
    def tile_beam_merge_with_batch(x, beam_size):
        """[B, ...] -> [B * beam, ...], each row repeated beam times (row b*beam+k is beam k of b)."""
        return _wrap(_t(x).repeat_interleave(beam_size, dim=0))

    def _split_batch_beams(self, x):
        t = _t(x)
        return t.reshape(-1, self.beam_size, *t.shape[1:])

    def _merge_batch_beams(self, x):
        t = _t(x)
        return t.reshape(-1, *t.shape[2:])

    def _gather(self, x, idx):
        """x [B, beam, ...] gathered along beams by idx [B, beam]."""
        t = _t(x)
        ix = idx.reshape(*idx.shape, *([1] * (t.dim() - 2))).expand(*idx.shape, *t.shape[2:])
        return t.gather(1, ix)

    # --------------------------------------------------------------------------- protocol
    def initialize(self, initial_cell_states):
        leaves = []
        _map(lambda a: leaves.append(_t(a)), initial_cell_states)
        ref = leaves[0]
        self.batch_size = ref.shape[0]
        cell_states = _map(lambda a: self.tile_beam_merge_with_batch(a, self.beam_size), initial_cell_states)
        B, K, dev = self.batch_size, self.beam_size, ref.device
        ids = torch.full((B, K), self.start_token, dtype=torch.int64, device=dev)
        inputs = self.embedding_fn(_wrap(ids)) if self.embedding_fn else _wrap(ids)
        log_probs = torch.full((B, K), -self.kinf, dtype=torch.float32, device=dev)
        log_probs[:, 0] = 0.0
        finished = torch.zeros((B, K), dtype=torch.bool, device=dev)
        lengths = torch.zeros((B, K), dtype=torch.int64, device=dev)
        state = self.StateWrapper(cell_states, _wrap(log_probs), _wrap(finished), _wrap(lengths))
        return inputs, state, _wrap(finished)

    def _beam_search_step(self, time, logits, next_cell_states, beam_state):
        lg = _t(logits).float()
        V = lg.shape[-1]
        step_lp = torch.log_softmax(lg, -1)
        fin = _t(beam_state.finished)
        # finished beams may only extend with end_token at zero cost
        noend = torch.full((V,), -self.kinf, dtype=step_lp.dtype, device=step_lp.device)
        noend[self.end_token] = 0.0
        step_lp = torch.where(fin.unsqueeze(-1), noend, step_lp)
        log_probs = step_lp + _t(beam_state.log_probs).unsqueeze(-1).to(step_lp.dtype)
        flat = log_probs.reshape(log_probs.shape[0], -1)
        top_scores, top_idx = flat.topk(self.beam_size, dim=-1)
        beam_idx = torch.div(top_idx, V, rounding_mode="floor")
        token = top_idx % V
        next_lp = flat.gather(1, top_idx)
        next_cell_states = _map(
            lambda s: _wrap(self._merge_batch_beams(self._gather(self._split_batch_beams(s), beam_idx))),
            next_cell_states)
        next_fin = self._gather(fin, beam_idx)
        next_len = self._gather(_t(beam_state.lengths), beam_idx) + (~next_fin).to(torch.int64)
        next_fin = next_fin | (token == self.end_token)
        out = self.OutputWrapper(_wrap(top_scores), _wrap(token), _wrap(beam_idx))
        state = self.StateWrapper(next_cell_states, _wrap(next_lp), _wrap(next_fin), _wrap(next_len))
        return out, state

    def step(self, time, inputs, states, **kwargs):
        merged_in = _map(lambda a: _wrap(self._merge_batch_beams(a)), inputs)
        cell_out, next_cell_states = self.cell(merged_in, states.cell_states, **kwargs)
        if self.output_fn is not None:
            cell_out = self.output_fn(cell_out)
        logits = self._split_batch_beams(cell_out)
        out, state = self._beam_search_step(time, logits, next_cell_states, states)
        nxt = self.embedding_fn(out.predicted_ids) if self.embedding_fn else out.predicted_ids
        return out, state, nxt, state.finished

    def finalize(self, outputs, final_states, sequence_lengths):
        return gather_tree(outputs.predicted_ids, outputs.parent_ids), final_states

    @property
    def tracks_own_finished(self):
        return True


def dynamic_decode(decoder, inits=None, max_step_num=None, output_time_major=False, impute_finished=False,
                   is_test=False, return_length=False, **kwargs):
    """Run ``decoder`` until every entry is finished or ``max_step_num`` steps were taken (reference
    decode.py:695).  -> (outputs, final_states[, sequence_lengths])."""
    inputs, states, finished = decoder.initialize(inits)
    fin = _t(finished)
    seq_len = torch.zeros(fin.shape, dtype=torch.int64, device=fin.device)
    steps = []
    step = 0
    while not bool(fin.all()):
        out, nstates, ninputs, nfin = decoder.step(_wrap(torch.tensor([step])), inputs, states, **kwargs)
        if not decoder.tracks_own_finished:
            nf = _t(nfin) | fin
            seq_len = seq_len + (~fin).to(torch.int64)
            if impute_finished:
                m = fin

                def keep(old, new):
                    o, n = _t(old), _t(new)
                    mm = m.reshape(*m.shape, *([1] * (n.dim() - m.dim())))
                    return _wrap(torch.where(mm, o, n))

                nstates = _map(keep, states, nstates)
            fin = nf
        else:
            seq_len = _t(getattr(nstates, "lengths", _wrap(seq_len)))
            fin = _t(nfin)
        steps.append(out)
        inputs, states = ninputs, nstates
        step += 1
        if max_step_num is not None and step > max_step_num:
            break
    outputs = _map(lambda *xs: _wrap(torch.stack([_t(x) for x in xs], 0)), *steps)
    final_states = states
    try:
        outputs, final_states = decoder.finalize(outputs, final_states, _wrap(seq_len))
    except NotImplementedError:
        pass
    if not output_time_major:
        outputs = _map(lambda x: _wrap(_t(x).transpose(0, 1)), outputs)
    res = (outputs, final_states)
    return res + (_wrap(seq_len),) if return_length else res
