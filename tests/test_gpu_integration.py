"""INTEGRATION.md is executable: its ctypes binding snippet and the C driver
(examples/decode_main.c) run on the GPU exactly as documented."""
import os
import re
import subprocess

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_integration_ctypes_snippet_runs(hip):
    text = open(os.path.join(REPO, "INTEGRATION.md")).read()
    code = re.search(r"## 3\. FFI binding.*?```python\n(.*?)```", text, re.S).group(1)
    cwd = os.getcwd()
    os.chdir(REPO)
    try:
        exec(compile(code, "INTEGRATION.md", "exec"), {})
    finally:
        os.chdir(cwd)


def test_c_driver_decodes(tmp_path):
    libdir = os.path.join(REPO, "llm.c-paged_amd")
    exe = str(tmp_path / "decode_main")
    subprocess.run(["gcc", "-O2", os.path.join(REPO, "examples", "decode_main.c"), "-I" + os.path.join(REPO, "include"),
                    "-L" + libdir, "-lpaged_hip", "-Wl,-rpath," + libdir, "-o", exe], check=True)
    r = subprocess.run([exe, "", "4", "6"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "tokens/s" in r.stdout
