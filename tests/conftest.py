import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")


def _ensure_built():
    """build when a library is missing, and rebuild when the library was built from other sources than
    this tree holds (fvhip_build_info's source hash): the tests never run a stale binary"""
    lib = os.path.join(ROOT, "fvens_amd", "libfvhip.so")
    orc = os.path.join(ROOT, "oracle", "liboracle.so")
    if not (os.path.exists(lib) and os.path.exists(orc)):
        import __graft_entry__
        __graft_entry__.build()
        return
    if os.environ.get("FVHIP_LIB"):
        return
    import subprocess
    import fvens_amd._ffi as ffi
    probe = subprocess.run([sys.executable, "-c", "import sys; sys.path.insert(0, %r); import fvens_amd._ffi as f; "
                            "print(f.lib().fvhip_build_info().decode())" % ROOT], capture_output=True, text=True)
    built = dict(x.split("=", 1) for x in probe.stdout.split() if "=" in x).get("src_sha256_16")
    if built != ffi.source_hash():
        sys.stderr.write("libfvhip.so was built from other sources (%s, tree %s): rebuilding\n" % (built, ffi.source_hash()))
        import __graft_entry__
        __graft_entry__.build()


_ensure_built()


@pytest.fixture(scope="session")
def gpu_available():
    import fvens_amd._ffi as ffi
    return ffi.lib().fvhip_device_count() > 0


def pytest_collection_modifyitems(config, items):
    # GPU tests fail loudly (not skip) when selected on a machine without a GPU: the product has no
    # CPU fallback. Without -m gpu they are deselected by the driver's -m "not gpu".
    pass


@pytest.fixture(autouse=True)
def _heartbeat(request):
    """a test that runs for minutes (the full-size partition and implicit tests) prints a line every 60 s
    past pytest's capture, so a watchdog that takes a silent run for a hung one sees it alive"""
    import threading
    import time
    done = threading.Event()
    t0 = time.time()

    capman = request.config.pluginmanager.getplugin("capturemanager")

    def beat():
        while not done.wait(60.0):
            line = "[heartbeat] %s running %.0f s\n" % (request.node.nodeid, time.time() - t0)
            if capman is None:
                sys.__stderr__.write(line)
                sys.__stderr__.flush()
                continue
            with capman.global_and_fixture_disabled():      # past pytest's fd capture
                sys.stderr.write(line)
                sys.stderr.flush()
    th = threading.Thread(target=beat, daemon=True)
    th.start()
    yield
    done.set()
