import os
import sys

# torch first: its HIP runtime (torch/lib/libamdhip64.so) is then the one
# liblzmagpu.so binds to, so tests that stage device buffers with torch and
# call the C ABI share one runtime.  Loaded the other way round, torch sees
# no device.
try:
    import torch  # noqa: F401
except ImportError:
    pass

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "lzma-sdk-zliblike_amd"))
