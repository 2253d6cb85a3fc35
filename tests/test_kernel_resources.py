"""Resource budget of the built gfx950 kernels (CPU-only: reads the code-object metadata).

A scratch spill inside a hot loop costs a memory round trip per use, and hipcc spills
silently (round 2 found 180 B of scratch in cnn_bwd's multi-image path), so every kernel
is pinned to zero scratch.  The LDS / register budgets pin the occupancy each kernel's
design assumes (docs/kernels.md).
"""
import glob
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = sorted(glob.glob(os.path.join(ROOT, "pytorch_distributed_mnist_amd", "_C*.so")))

pytestmark = pytest.mark.skipif(
    not SO or not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-readelf"),
    reason="extension not built or ROCm llvm tools absent")


@pytest.fixture(scope="module")
def kernels():
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from kernel_resources import kernels as read
    ks = read(SO[0])
    assert ks, "no kernels found in the extension's code objects"
    return ks


def _find(ks, name):
    hits = {k: v for k, v in ks.items() if name in k}
    assert hits, f"kernel {name} not found"
    return hits


def test_no_kernel_uses_scratch(kernels):
    spilled = {k: v["private_segment_fixed_size"] for k, v in kernels.items()
               if v.get("private_segment_fixed_size", 0) != 0}
    assert not spilled, f"kernels with scratch: {spilled}"


def test_every_hot_kernel_is_present(kernels):
    for name in ("cnn_fwd_kernel", "fc1_fwd_kernel", "cnn_head_kernel", "fc1_bwd_kernel",
                 "cnn_bwd_kernel", "conv_reduce_kernel", "optim_kernel", "lin_train_kernel",
                 "xgmi_allreduce_kernel", "cnn_fwd_band_kernel", "cnn_bwd_band_kernel"):
        _find(kernels, name)


def test_occupancy_budgets(kernels):
    # cnn_bwd: one 512-thread workgroup per CU (its LDS carve), <= 256 registers per lane
    for k, v in _find(kernels, "cnn_bwd_kernel").items():
        assert v["group_segment_fixed_size"] <= 163840, k
        assert v["vgpr_count"] + v.get("agpr_count", 0) <= 256, k
    # cnn_fwd: two 512-thread workgroups per CU (<= 80 KB LDS, <= 128 registers)
    for k, v in _find(kernels, "cnn_fwd_kernel").items():
        assert v["group_segment_fixed_size"] <= 81920, k
        assert v["vgpr_count"] + v.get("agpr_count", 0) <= 128, k
    # small-batch row-band kernels: cnn_fwd_band two 512-thread workgroups per CU,
    # cnn_bwd_band one (<= 256 registers per lane), both within the 160 KB LDS
    for k, v in _find(kernels, "cnn_fwd_band_kernel").items():
        assert v["group_segment_fixed_size"] <= 81920, k
        assert v["vgpr_count"] + v.get("agpr_count", 0) <= 128, k
    for k, v in _find(kernels, "cnn_bwd_band_kernel").items():
        assert v["group_segment_fixed_size"] <= 163840, k
        assert v["vgpr_count"] + v.get("agpr_count", 0) <= 256, k
    # fc1_bwd (and the fp32 program's): 256 threads, at most one wave per SIMD each
    for k, v in _find(kernels, "fc1_bwd_kernel").items():
        assert v["vgpr_count"] + v.get("agpr_count", 0) <= 512, k


def _alloc(v):
    return -(-(v["vgpr_count"] + v.get("agpr_count", 0)) // 8) * 8


def test_collective_kernels_fit_beside_cnn_bwd(kernels):
    """The xgmi collectives run beside cnn_bwd, which takes 163,200 of a CU's 163,840 LDS
    bytes: any LDS allocation of theirs would keep cnn_bwd's workgroup off their CUs for the
    whole persistent launch (two rounds of cnn_bwd, 17 -> 30 us at B = 256).  They use none,
    and few enough registers to share a SIMD with the two waves of the backward kernel they run
    beside (512 per lane, allocated in blocks of 8): the narrow persistent kernel beside the
    one-image cnn_bwd and every band kernel, the wide one beside the 4- and 8-row bands."""
    def free(pred):
        ks = [v for k, v in kernels.items() if pred(k)]
        assert ks
        return min(512 - 2 * _alloc(v) for v in ks)
    every = free(lambda k: "cnn_bwd_band_kernel" in k or ("cnn_bwd_kernel" in k and "ILb1E" in k))
    small = free(lambda k: "cnn_bwd_band_kernelILi4E" in k or "cnn_bwd_band_kernelILi8E" in k)
    for name in ("xgmi_stream_kernel", "xgmi_allreduce_kernel", "xgmi_wait_kernel"):
        for k, v in _find(kernels, name).items():
            assert v["group_segment_fixed_size"] == 0, k
            limit = small if "ILi8E" in k else every
            assert _alloc(v) <= limit, (k, _alloc(v), limit)


def test_fc1_bwd_two_workgroups_per_cu(kernels):
    """fc1_bwd runs two 256-thread workgroups per CU (its 503 workgroups at B = 256 in one
    round): <= 256 registers per lane and two LDS carves."""
    for k, v in _find(kernels, "fc1_bwd_kernelEPKDF16b").items():
        assert _alloc(v) <= 256, (k, _alloc(v))
        assert 2 * v["group_segment_fixed_size"] <= 163840, k
