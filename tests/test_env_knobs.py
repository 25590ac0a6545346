"""The diagnostics knobs of docs/ENVIRONMENT.md: CNMF_LOG_LEVEL sets the package logger's
level (utils/log.py); CNMF_TRACE=1 prints each timed stage (utils/timing.py)."""
import logging
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _child(code: str, **env) -> str:
    e = dict(os.environ, **env)
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=e, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout


@pytest.mark.parametrize("level", ["DEBUG", "ERROR"])
def test_log_level_from_environment(level):
    out = _child("import logging; from cnmf_torch_amd.utils.log import get_logger; "
                 "print(get_logger().getEffectiveLevel())", CNMF_LOG_LEVEL=level)
    assert int(out.strip()) == getattr(logging, level)


def test_trace_prints_each_stage():
    code = ("from cnmf_torch_amd.utils.timing import StageTimer\n"
            "t = StageTimer()\n"
            "with t('prepare'):\n    pass\n"
            "with t('factorize'):\n    pass\n"
            "print(sorted(t.summary()))\n")
    on = _child(code, CNMF_TRACE="1")
    assert "[cnmf trace] prepare:" in on and "[cnmf trace] factorize:" in on
    off = _child(code, CNMF_TRACE="0")
    assert "[cnmf trace]" not in off and "['factorize', 'prepare']" in off
