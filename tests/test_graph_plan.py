"""The graphs prepare() captures cover every replay train_steps() makes, and no more
(runtime/gpu_step.py _plan / _variants; CPU only: nothing is captured)."""
import pytest

from pytorch_distributed_mnist_amd.runtime.gpu_step import GpuStepBase


def _step(carries: bool, graph_steps: int = 8, period: int = 2):
    st = GpuStepBase.__new__(GpuStepBase)
    st.GRAPH_STEPS = graph_steps
    st.GRAPH_SIZES = tuple(range(graph_steps, 0, -1))
    st.phase_period = period
    st.carries_across_graphs = lambda B: carries
    return st


@pytest.mark.parametrize("carries", [False, True])
@pytest.mark.parametrize("graph_steps", [1, 2, 5, 8, 16])
def test_prepared_graphs_are_exactly_the_replayed_ones(carries, graph_steps):
    st = _step(carries, graph_steps)
    prepared = set(st._variants(256, st.GRAPH_SIZES))
    replayed = set()
    for n in range(1, 5 * graph_steps + 3):
        for start_phase in range(st.phase_period):
            ph = start_phase
            plan = st._plan(256, n)
            assert sum(s for s, _, _ in plan) == n
            for size, ci, co in plan:
                replayed.add((size, ph, ci, co))
                ph = (ph + size) % st.phase_period
    assert replayed <= prepared, replayed - prepared
    assert prepared == replayed, prepared - replayed


def test_carrying_plan_hands_the_update_between_replays():
    st = _step(True)
    assert st._plan(256, 19) == [(8, False, True), (8, True, True), (3, True, False)]
    assert st._plan(256, 1) == [(1, False, False)]
    assert _step(False)._plan(256, 9) == [(8, False, False), (1, False, False)]
    assert _step(True, 16)._plan(256, 10) == [(10, False, False)]
