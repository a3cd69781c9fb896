import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT / "scenery-insitu_amd", ROOT / "tests", ROOT):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libinsitu_hip.so)")
    config.addinivalue_line("markers", "slow: larger CPU oracle cases")


def pytest_collection_modifyitems(config, items):
    # GPU tests fail loudly when no GPU is present; they are only selected with -m gpu.
    pass
