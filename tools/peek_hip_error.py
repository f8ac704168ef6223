"""pytest plugin (diagnostic): after each test, report a pending HIP error (hipPeekAtLastError)
so a test that leaves one behind is named.  usage: PYTHONPATH=tools pytest -p peek_hip_error"""
import ctypes

_hip = None


def pytest_runtest_teardown(item, nextitem):
    global _hip
    if _hip is None:
        _hip = ctypes.CDLL('libamdhip64.so')
    rc = _hip.hipPeekAtLastError()
    if rc:
        print(f'\n[peek] {item.nodeid}: pending HIP error {rc}', flush=True)
