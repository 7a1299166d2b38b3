import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs under gpurun on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def native():
    import torch  # noqa: F401  (before the native lib, see _native docstring)
    from mipipe import _native
    _native.build()
    return _native.lib()


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.fixture(scope="session")
def model_dir(tmp_path_factory):
    return tmp_path_factory.mktemp("models")


def make_model(model_dir, name, ftype, seed=0, **kw):
    from mipipe.models.config import CONFIGS
    from mipipe.models.synthetic import write_synthetic_gguf
    cfg = CONFIGS[name]
    if kw:
        cfg = cfg.scaled(**kw)
    path = os.path.join(str(model_dir), f"{cfg.name}-{ftype}-{seed}-{abs(hash(tuple(sorted(kw.items()))))}.gguf")
    if not os.path.exists(path):
        write_synthetic_gguf(path, cfg, ftype, seed=seed, fast_random_blocks=False, wscale=1.0)
    return path, cfg
