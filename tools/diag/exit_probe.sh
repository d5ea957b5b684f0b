#!/bin/bash
# Round-3 verdict, weak 3: a SIGSEGV at process exit under rocprofv3 (gpurun_out/r3b/bench_c2.log).  Round 4 saw it
# again with no torch in the process (gpurun_out/r4b/bench_c2.log).  The probes run from the least to the most of our
# code in the process and the script stops at the first one that does not exit cleanly (a crashed process ends the
# GPU work of the call).  Each prints its exit code.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4i/exit; mkdir -p $O
P="import sys; sys.path.insert(0, '$R'); from gameoflifewithactors_amd import _lib, Board; _lib.load()"
probe() {  # probe NAME PYCODE: under rocprofv3 --kernel-trace --stats; stops the script unless it exits 0
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$1 -o run -- python3 -c "$2" > $O/$1.log 2>&1
  local rc=$?
  echo "$1 rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $O/$1.log; exit $rc; fi
}
# Round 4, first call (gpurun_out/r4h/exit): a minimal hipcc library dlclosed before exit exits clean; a
# cooperative board with libgol_hip.so dlclosed before exit still crashes in the same frames -- so not our module
# destructors.  Next: the cooperative launch (the runtime's cooperative queue, torn down after the profiler).
# 1. the cooperative pass launched with hipLaunchKernel (board option coop_launch 0), library unloaded
probe coop_plain_unload "$P
with Board(4096, 4096, 0, options={'coop_launch': 0}) as b: b.seed_splitmix(1).step(100); b.synchronize()
_lib.unload()"
# 2. the same without the unload
probe coop_plain "$P
with Board(4096, 4096, 0, options={'coop_launch': 0}) as b: b.seed_splitmix(1).step(100); b.synchronize()"
# 3. a streaming board (no persistent pass)
probe stream_board "$P
with Board(65536, 4096, 0) as b: b.seed_splitmix(1).step(24); b.synchronize()"
# 4. the smallest hipcc library with one kernel (not libgol_hip.so), loaded by ctypes, no dlclose
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -shared -fPIC -o $O/libtiny.so $R/tools/diag/tiny.hip || exit 1
probe tiny_lib "import ctypes; l = ctypes.CDLL('$O/libtiny.so'); print('tiny', l.tiny_run())"
# 5. a cooperative board (bench_c2's pass, cooperative launch)
probe coop_board "$P
with Board(4096, 4096, 0) as b: b.seed_splitmix(1).step(100); b.synchronize()"
