"""One HIP runtime per process ("two HIP runtimes collide"; ADVICE round 3, no torch import as a
side effect of loading the library).

torch bundles its own libamdhip64 (ROCm 7.0) under the soname libgol_hip.so links against (/opt/rocm, 7.2), and the
loader binds every later library to whichever came first.  The rule (`_lib._torch_runtime_first`): a process that
uses torch imports it before the library and both share torch's runtime; a process without torch (the F# host, the
C++ mirror, bench.py's handle leg) runs the library on /opt/rocm's runtime; importing torch AFTER the library loaded
its own runtime warns with the explanation instead of leaving torch to fail at its first kernel.  Each case runs in a fresh
child process; the same board gives the same hash under both runtimes.
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
_TORCH_LATE = """
import warnings
with warnings.catch_warnings(record=True) as caught:
    warnings.simplefilter("always")
    import torch
out["late_torch"] = [str(w.message) for w in caught if issubclass(w.category, RuntimeWarning)]
"""


def _run(parts):
    code = "import json, sys\nsys.path.insert(0, %r)\nout = {}\n" % ROOT
    code += "".join(parts)
    code += ("from gameoflifewithactors_amd import _lib\nout['runtimes'] = _lib.hip_runtimes()\n"
             "print(json.dumps(out))\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_torch_first_shares_torchs_runtime_and_library_alone_runs_on_rocm():
    shared = _run(["import torch\n", _BOARD, _STRIPS])
    assert len(shared["runtimes"]) == 1 and "/torch/" in shared["runtimes"][0], shared
    assert shared["board"] == shared["strips"], shared  # same board, same 24 generations, both paths
    alone = _run([_BOARD])
    assert len(alone["runtimes"]) == 1 and "/torch/" not in alone["runtimes"][0], alone
    assert alone["board"] == shared["board"], (alone, shared)  # the same result under /opt/rocm's runtime


def test_torch_after_the_library_warns():
    out = _run([_BOARD, _TORCH_LATE])
    assert any("import torch before" in m for m in out["late_torch"]), out
    # what the warning is about: torch then maps its own runtime beside the library's (two are mapped now)
    assert len(out["runtimes"]) == 2 and any("/torch/" not in r for r in out["runtimes"]), out
