"""The C oracle under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md §5 sanitizer row).

`make -C oracle sanitize` builds oracle/sanitize_main.c with the oracle sources (-fsanitize=address,undefined,
-fno-sanitize-recover=all, leak detection on) and drives every mgo_opts option on small 2D / 3D, cubic and
non-cubic boxes, the stateless per-level functions and twoGrid.  Any sanitizer report fails the run.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None and shutil.which("cc") is None, reason="no C compiler")
def test_oracle_clean_under_asan_ubsan():
    p = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "sanitize"], capture_output=True, text=True,
                       timeout=600)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert "sanitize ok" in p.stdout
