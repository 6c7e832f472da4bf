"""The key directory's probe keeps its long-key tail compare out of line
(k_keys.hip:102-113): compiled for gfx950, k_key_probe must CALL
key_tail_equal rather than inline it.  Round 5 found the inlined form losing
the matched slot on keys over 16 bytes (every such key re-created on every
call); tools/mc_keyprobe.hip reproduces that loop shape standalone, inlined
and out of line, on the GPU (profiles/r06_mc_keyprobe.log).  This test needs
only hipcc (a device-only compile to assembly, ~2 s), no GPU."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _asm(tmp_path, src):
    out = tmp_path / "k.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-S", "-w",
                    "-o", str(out), os.path.join(ROOT, "jylis_amd", "csrc", src)], check=True,
                   stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    return out.read_text()


def _body(asm, fn_substr):
    m = re.search(r"^(_Z\S*" + fn_substr + r"\S*):", asm, re.M)
    assert m, fn_substr
    start = m.end()
    end = asm.index("s_endpgm", start)
    return asm[start:end]


@pytest.mark.skipif(not (os.path.exists(HIPCC) or shutil.which("hipcc")), reason="needs hipcc")
def test_key_probe_calls_the_tail_compare(tmp_path):
    asm = _asm(tmp_path, "k_keys.hip")
    # the tail compare is its own function ...
    assert re.search(r"^_Z\S*key_tail_equal\S*:", asm, re.M)
    body = _body(asm, "k_key_probe")
    # ... and the probe loop reaches it through a call
    assert "s_swappc_b64" in body
    assert "key_tail_equal" in body
