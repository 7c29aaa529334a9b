"""pytest configuration: the ``gpu`` marker and import paths.

``oracle/`` is test infrastructure (CPU restatement of the reference); the
product package lives in ``rs-bann_amd/`` (hyphenated directory, so it is put on
sys.path and imported as ``bann``).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "rs-bann_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
