"""CPU: host-only AddressSanitizer + UndefinedBehaviorSanitizer build of the C++ host units
that read untrusted input or do wide integer arithmetic -- hmm_json.cpp (malformed files,
every truncation of a valid file, random byte flips), csp.cpp (exact term accumulation, the
limb-carry search vs brute force) and exact_fixed.h (f32/f64 limbs vs an __int128 reference)
-- driven by tools/sanitize/san_driver.cpp.  Never built or run on the GPU box."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

SAN = os.path.join(ROOT, "tools", "sanitize")


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("make") is None, reason="needs g++ and make")
def test_host_units_under_asan_ubsan():
    r = subprocess.run(["make", "-s", "-C", SAN, "run"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "all checks passed" in r.stdout
