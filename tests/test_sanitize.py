"""Host-side ASan + UBSan pass over the C++ runtime (tools/sanitize.sh): the scheduler,
tag and two-process remote-edge cases must finish with no sanitizer report (memory
errors, undefined behaviour or leaks such as ownership cycles between ports, blocks and
schedulers). CPU only; GPU sanitizers are not available on the MI355X pool."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _asan_available():
    if shutil.which("g++") is None:
        return False
    r = subprocess.run(["g++", "-print-file-name=libasan.so"], capture_output=True, text=True)
    return r.returncode == 0 and os.path.sep in r.stdout.strip()


@pytest.mark.skipif(not _asan_available(), reason="g++ with libasan needed")
def test_runtime_clean_under_asan_ubsan(tmp_path):
    env = dict(os.environ, OUT=str(tmp_path / "asan"))
    r = subprocess.run([os.path.join(ROOT, "tools", "sanitize.sh")], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=1200)
    logs = ""
    for f in sorted((tmp_path / "asan").glob("*.log")):
        logs += f"--- {f.name}\n" + f.read_text()[-4000:]
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:] + logs
