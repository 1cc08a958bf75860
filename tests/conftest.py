import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "geth-sharding_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built libgsv.so")


# extra flags for the host builds of device headers / host decoders (tests/native): set by
# tools/sanitize.sh, which also preloads the ASan/UBSan runtimes into the Python process
SANITIZE_FLAGS = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
                  "-fno-sanitize-recover=undefined"] if os.environ.get("GSV_SANITIZE") == "1" else []


def build_native(src, out, std="c++17", defines=()):
    """g++ -shared of tests/native/<src> (plus the sanitizer flags when GSV_SANITIZE=1)."""
    import subprocess
    subprocess.run(["g++", "-O2", f"-std={std}", "-shared", "-fPIC", "-Wno-unknown-pragmas"] + SANITIZE_FLAGS +
                   [f"-D{d}" for d in defines] +
                   ["-o", str(out), os.path.join(os.path.dirname(os.path.abspath(__file__)), "native", src)],
                   check=True)
    import ctypes
    return ctypes.CDLL(str(out))


def golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.lib()
    return O


@pytest.fixture(scope="session")
def ctx():
    """The product context on the GPU (fails loudly if libgsv.so or the GPU is missing)."""
    import gsv
    return gsv.default_context()
