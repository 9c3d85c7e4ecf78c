import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'tests', 'golden')):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (HIP extension, cuda:0)')


import gc  # noqa: E402

import pytest  # noqa: E402


@pytest.fixture(autouse=True)
def _release_device_memory():
    """After every test: drop the test's tensors and hand the caching allocator's blocks back to
    the device. The real-size C3 / C5 tests leave ~100 GB cached in this process otherwise, which
    the multi-process tests' spawned ranks (their own allocators, the same GPU) then cannot get."""
    yield
    import torch
    if torch.cuda.is_initialized():
        gc.collect()
        torch.cuda.empty_cache()


# Heartbeat for long tests (the C5 configured-batch oracle test runs its CPU oracle for minutes
# with its output captured): a daemon thread reports, every 60 s of one test, the test's id and
# elapsed time on the terminal and in gpurun_out/pytest_heartbeat.txt, so a run watched for
# silence is not taken for a hung one.
import threading  # noqa: E402
import time  # noqa: E402

_HB = {'test': None, 't0': 0.0, 'tr': None}


def _heartbeat():
    path = os.path.join(ROOT, 'gpurun_out', 'pytest_heartbeat.txt')
    while True:
        time.sleep(60)
        test, t0 = _HB['test'], _HB['t0']
        if test is None or time.time() - t0 < 55:
            continue
        msg = f'[heartbeat] {test} running {time.time() - t0:.0f} s'
        try:
            os.makedirs(os.path.dirname(path), exist_ok=True)
            with open(path, 'a') as f:
                f.write(msg + '\n')
        except OSError:
            pass
        tr = _HB['tr']
        if tr is not None:
            try:
                tr.write_line(msg)
            except Exception:  # the reporter is not thread-safe; the file carries the beat
                pass


def pytest_sessionstart(session):
    _HB['tr'] = session.config.pluginmanager.get_plugin('terminalreporter')
    threading.Thread(target=_heartbeat, name='pytest-heartbeat', daemon=True).start()


def pytest_runtest_logstart(nodeid, location):
    _HB['test'], _HB['t0'] = nodeid, time.time()


def pytest_runtest_logfinish(nodeid, location):
    _HB['test'] = None
