"""One HIP runtime per process, whatever the import order ("two HIP runtimes collide").

torch bundles its own libamdhip64 under the soname libgol_hip.so links against (/opt/rocm).  `_lib.load()` puts
torch's runtime in first whenever torch is importable; these tests run each order once in a fresh child process
(the C-ABI board first, then the torch strip runner; and the reverse) and check both work on one runtime.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_BOARD = """
from gameoflifewithactors_amd import Board
with Board(4096, 512, 0, options={"coop": 0}) as b:
    b.seed_splitmix(7).step(24)
    out["board"] = b.hash()
"""
_STRIPS = """
import torch
from gameoflifewithactors_amd.strips import StripRunner
r = StripRunner(4096, 512, 0, 12, device=torch.device("cuda", 0))
r.seed_splitmix(7)
r.step_pass(); r.step_pass()
torch.cuda.synchronize()
out["strips"] = r.hash()
"""


@pytest.mark.parametrize("order", [("board", "strips"), ("strips", "board")])
def test_import_order_shares_one_runtime(order):
    code = "import json, sys\nsys.path.insert(0, %r)\nout = {}\n" % ROOT
    for part in order:
        code += _BOARD if part == "board" else _STRIPS
    code += ("from gameoflifewithactors_amd import _lib\nout['runtimes'] = _lib.hip_runtimes()\n"
             "print(json.dumps(out))\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert len(out["runtimes"]) == 1, out
    assert out["board"] == out["strips"], out  # same board, same 24 generations, both paths
