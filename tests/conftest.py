import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libxdrgpu.so on cuda:0)")
    config.addinivalue_line("markers", "slow: full BASELINE-size cases")


@pytest.fixture(scope="session")
def gpu_ctx():
    import torch
    from oncrpc4j_amd import engine
    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a visible GPU")
    ctx = engine.Context(0)
    ctx.set_stream(torch.cuda.current_stream())
    yield ctx
    ctx.close()
