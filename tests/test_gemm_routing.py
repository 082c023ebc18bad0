"""Route selection of the native GEMM entry points (ops/gemm.py), checked on CPU by recording what each pass would
launch: the forward on W as stored (V7_NNF) with its tile-group rule, the weight gradient's persistent MN-major
kernel for a first write and v4's kernel for accumulation, and the env overrides."""
import torch

from paddle2_amd.ops import gemm as G


def _record(monkeypatch):
    calls = []

    def fake_launch(layout, epi, a, lda, b, ldb, c, ldc, c2, ldc2, bias, M, Nn, K, beta=0.0, H=0, name="fwd"):
        calls.append(dict(layout=layout, epi=epi, M=M, N=Nn, K=K, beta=beta, name=name, variant=G._variant(name),
                          group=G.GROUP_M if G._GROUP_FORCED else G.PASS_GROUP_M.get(name, G.GROUP_M),
                          b_ptr=b.data_ptr()))

    monkeypatch.setattr(G, "_launch", fake_launch)
    monkeypatch.setattr(G, "VARIANT", None)
    return calls


def test_forward_runs_on_w_as_stored(monkeypatch):
    calls = _record(monkeypatch)
    x = torch.zeros(32768, 4096, dtype=torch.bfloat16)
    for n, group in ((12288, 4), (22016, 2), (32000, 2)):
        w = torch.zeros(4096, n, dtype=torch.bfloat16)
        G.mm_fwd(x, w)
        c = calls[-1]
        assert c["layout"] == G.LAYOUT_AK and c["variant"] == G.V7_NNF and c["group"] == group
        assert c["b_ptr"] == w.data_ptr()          # W itself, no transposed copy
    # short token batches keep group 4 even for wide outputs
    G.mm_fwd(torch.zeros(4096, 5120, dtype=torch.bfloat16), torch.zeros(5120, 20480, dtype=torch.bfloat16))
    assert calls[-1]["name"] == "fwd_nn" and calls[-1]["group"] == 4


def test_forward_tn_route_when_disabled(monkeypatch):
    calls = _record(monkeypatch)
    monkeypatch.setattr(G, "FWD_NN_MAX_M", 0)
    monkeypatch.setattr(G, "_wt", lambda w: w.t().contiguous())
    x, w = torch.zeros(512, 256, dtype=torch.bfloat16), torch.zeros(256, 768, dtype=torch.bfloat16)
    G.mm_fwd(x, w)
    c = calls[-1]
    assert c["layout"] == G.LAYOUT_AK | G.LAYOUT_BK and c["variant"] == G.V7_SPREAD and c["b_ptr"] != w.data_ptr()


def test_weight_gradient_routes(monkeypatch):
    calls = _record(monkeypatch)
    x = torch.zeros(32768, 4096, dtype=torch.bfloat16)
    dy = torch.zeros(32768, 12288, dtype=torch.bfloat16)
    out = torch.zeros(4096, 12288)
    G.mm_wgrad(x, dy, out, beta=0.0)          # first write: persistent MN-major kernel, group 8
    assert calls[-1]["variant"] == G.V7_MN and calls[-1]["layout"] == 0 and calls[-1]["group"] == 8
    G.mm_wgrad(x, dy, out, beta=1.0)          # accumulation: v4's read-modify-write kernel
    assert calls[-1]["name"] == "wgrad_acc" and calls[-1]["variant"] == 5
    xs, dys = torch.zeros(4096, 5120, dtype=torch.bfloat16), torch.zeros(4096, 15360, dtype=torch.bfloat16)
    G.mm_wgrad(xs, dys, torch.zeros(5120, 15360), beta=0.0)   # short tokens into a wide output: group 4
    assert calls[-1]["name"] == "wgrad_short" and calls[-1]["variant"] == G.V7_MN and calls[-1]["group"] == 4


def test_variant_override_disables_the_n_major_forward(monkeypatch):
    _record(monkeypatch)
    monkeypatch.setattr(G, "VARIANT", 5)
    assert not G._fwd_nn(4096)
    monkeypatch.setattr(G, "VARIANT", None)
    assert G._fwd_nn(4096)
    monkeypatch.setenv("PADDLE2_AMD_GEMM_VARIANT_FWD", "6")
    assert not G._fwd_nn(4096)
