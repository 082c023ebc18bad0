"""Host-side split-K planning of the <= 16-row decode GEMM (csrc/kernels/weight_only.hip pd_wo_splits): the 768
workgroup target picked in profiles/r6_decode_partials.md, checked on CPU through the extension's host function."""
import os

import pytest

from paddle2_amd.ops import _native as N

C = N.native()
pytestmark = pytest.mark.skipif(C is None or "PADDLE2_AMD_DEC_WG_TARGET" in os.environ,
                                reason="native extension not built / target overridden")


@pytest.mark.parametrize("n,k,splits", [(4096, 4096, 12), (12288, 4096, 4), (22016, 4096, 3), (4096, 11008, 12),
                                        (32000, 4096, 2)])
def test_llama7b_decode_split_counts(n, k, splits):
    for m in (1, 8, 16):
        assert C.dec_splits(m, n, k) == splits


def test_splits_reach_the_workgroup_target_and_stay_within_k():
    for n, k in ((4096, 4096), (12288, 4096), (4096, 11008), (1024, 512)):
        s = C.dec_splits(1, n, k)
        assert 1 <= s <= k // 64
        assert s * (n // 64) >= 768 or s == k // 64
