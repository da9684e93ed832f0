import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP (MI355X) device")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def _has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no HIP device visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def gpu():
    import torch
    return torch.device("cuda", 0)


@pytest.fixture(scope="session")
def small_data(tmp_path_factory):
    """Synthetic 50-stock panel taken through L0 -> L2 -> L3 once per session (CPU)."""
    from pfml.config import Config
    from pfml.data import synthetic as syn, acquire
    from pfml.models import prep, risk
    d = str(tmp_path_factory.mktemp("pfml_small"))
    spec = syn.small_spec()
    syn.write_raw(syn.generate(spec), d)
    cfg = syn.settings_for_small(Config.default().override([f"run.data_dir={d}"]), spec)
    acquire.get_additional_data(cfg)
    acquire.sp500_subset(cfg)
    prep.prepare_data(cfg)
    risk.estimate_cov(cfg)
    return cfg
