#!/bin/bash
# Round-3 verdict, weak 3: a SIGSEGV at process exit under rocprofv3 (gpurun_out/r3b/bench_c2.log).  Round 4 saw it
# again with no torch in the process (gpurun_out/r4b/bench_c2.log).  Each probe prints its exit code.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4f/exit; mkdir -p $O
P="import sys; sys.path.insert(0, '$R'); from gameoflifewithactors_amd import _lib, Board; _lib.load()"
probe() {  # probe NAME PYCODE [under-profiler]
  if [ "$3" = prof ]; then
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$1 -o run -- python3 -c "$2" > $O/$1.log 2>&1
  else
    timeout -k 10 120 python3 -c "$2" > $O/$1.log 2>&1
  fi
  echo "$1 rc=$?"
}
probe load_only_prof "$P" prof
probe stream_board_prof "$P
with Board(65536, 4096, 0) as b: b.seed_splitmix(1).step(24); b.synchronize()" prof
probe coop_board_prof "$P
with Board(4096, 4096, 0) as b: b.seed_splitmix(1).step(100); b.synchronize()" prof
probe coop_board_noprof "$P
with Board(4096, 4096, 0) as b: b.seed_splitmix(1).step(100); b.synchronize()"
probe coop_board_prof_os_exit "$P
import os
with Board(4096, 4096, 0) as b: b.seed_splitmix(1).step(100); b.synchronize()
sys.stdout.flush(); os._exit(0)" prof
probe torch_then_coop_prof "import torch; $P
with Board(4096, 4096, 0) as b: b.seed_splitmix(1).step(100); b.synchronize()" prof
# the smallest hipcc library with one kernel (not libgol_hip.so): built here, loaded by ctypes
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -shared -fPIC -o $O/libtiny.so $R/tools/diag/tiny.hip && \
probe tiny_lib_prof "import ctypes; l = ctypes.CDLL('$O/libtiny.so'); print('tiny', l.tiny_run())" prof
probe tiny_lib_noprof "import ctypes; l = ctypes.CDLL('$O/libtiny.so'); print('tiny', l.tiny_run())"
