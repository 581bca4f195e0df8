"""Static guard: no undefined names in the product, bench and tool sources (tools/lint_names.py)."""
import os
import subprocess
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def test_no_undefined_names():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "lint_names.py")], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
