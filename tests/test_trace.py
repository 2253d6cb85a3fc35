"""roctx tracing helper (utils/trace.py): a no-op when disabled, nesting ranges when on."""
from pytorch_distributed_mnist_amd.utils import trace


def test_trace_ranges_nest_and_disable():
    was = trace.enabled()
    try:
        trace.enable(False)
        with trace.range("off"):
            pass
        on = trace.enable(True)          # False only if libroctx64 is absent
        assert on == trace.enabled()
        with trace.range("outer"):
            with trace.range("inner"):
                trace.mark("point")
    finally:
        trace.enable(was)
