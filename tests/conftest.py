import importlib.util
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "video-stream-segmenetation_amd")
sys.path.insert(0, os.path.join(ROOT, "oracle"))  # tests may import the oracle (checker)


def load_pkg():
    """The package directory name is not an identifier; load it as `vss_amd`."""
    if "vss_amd" in sys.modules:
        return sys.modules["vss_amd"]
    spec = importlib.util.spec_from_file_location("vss_amd", os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["vss_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")


@pytest.fixture(scope="session")
def pkg():
    return load_pkg()


@pytest.fixture(scope="session")
def blob(pkg):
    path = pkg.ensure_weights()
    with open(path, "rb") as f:
        return f.read()


@pytest.fixture(scope="session")
def synthetic(pkg):
    import vss_amd.synthetic as s  # noqa: F401
    return sys.modules["vss_amd.synthetic"]


@pytest.fixture(scope="session")
def oracle():
    import oracle_py
    oracle_py.build()
    return oracle_py
