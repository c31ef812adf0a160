import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


# The tests exercise the library's and the engine's tuning knobs (tiling, MT19937 chain layout,
# streams, cache budget) on purpose; production reads none of them without this switch
# (spgg_abi.h "Environment knobs", engine.tuning_env).
os.environ.setdefault("SPGG_TUNING", "1")
