import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a MI355X (runs through libtmatch on the device)")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session", autouse=True)
def _built():
    from emqx_amd import build
    build.build_work()
    build.build_oracle()
    if os.environ.get("TM_SKIP_HIP_BUILD") != "1" and build.LIB_TMATCH.exists() is False:
        build.build_tmatch()
    yield
