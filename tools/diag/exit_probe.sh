#!/bin/bash
# Round-3 verdict, weak 3: a SIGSEGV at process exit under rocprofv3 (gpurun_out/r3b/bench_c2.log).  Round 4 saw it
# again with no torch in the process (gpurun_out/r4b/bench_c2.log).  The probes run from the least to the most of our
# code in the process and the script stops at the first one that does not exit cleanly (a crashed process ends the
# GPU work of the call).  Each prints its exit code.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4h/exit; mkdir -p $O
P="import sys; sys.path.insert(0, '$R'); from gameoflifewithactors_amd import _lib, Board; _lib.load()"
probe() {  # probe NAME PYCODE: under rocprofv3 --kernel-trace --stats; stops the script unless it exits 0
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$1 -o run -- python3 -c "$2" > $O/$1.log 2>&1
  local rc=$?
  echo "$1 rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $O/$1.log; exit $rc; fi
}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -shared -fPIC -o $O/libtiny.so $R/tools/diag/tiny.hip || exit 1
T="import ctypes, _ctypes; l = ctypes.CDLL('$O/libtiny.so'); print('tiny', l.tiny_run())"
# 0. dlclose before exit (the library's device code unregistered while the profiler is alive): expected clean
probe tiny_lib_dlclose "$T
_ctypes.dlclose(l._handle)"
probe coop_board_unload "$P
with Board(4096, 4096, 0) as b: b.seed_splitmix(1).step(100); b.synchronize()
_lib.unload()"
# 1. the smallest hipcc library with one kernel (not libgol_hip.so), loaded by ctypes
probe tiny_lib "$T"
# 2. libgol_hip.so loaded, no board
probe load_only "$P"
# 3. a streaming board
probe stream_board "$P
with Board(65536, 4096, 0) as b: b.seed_splitmix(1).step(24); b.synchronize()"
# 4. a cooperative board (bench_c2's pass)
probe coop_board "$P
with Board(4096, 4096, 0) as b: b.seed_splitmix(1).step(100); b.synchronize()"
