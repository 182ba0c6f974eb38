#!/bin/bash
# Build an A/B baseline library: the current objects, with the named sources taken from a git rev.
# usage: scripts/build_ab.sh <rev> <src.hip> [...]   -> ab/_C_base.so  (load with RDP_NATIVE_SO)
set -e
cd "$(dirname "$0")/.."
rev=$1; shift
python -m robotic_discovery_platform_amd._build > /dev/null
mkdir -p ab build/ab
objs=""
for o in build/obj/*.o; do objs="$objs $o"; done
for src in "$@"; do
  git show "$rev:csrc/$src" > build/ab/$src
  case $src in
    *.hip) /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=fast -munsafe-fp-atomics -I csrc -c build/ab/$src -o build/ab/$src.o ;;
    *.cpp) python - "$src" <<'PY'
import os, subprocess, sys, sysconfig
from robotic_discovery_platform_amd import _build as b
src = sys.argv[1]
tinc, _, abi = b._torch_paths()
cmd = ["g++", "-O3", "-fPIC", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-DUSE_ROCM", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
       "-I", b.CSRC, "-I", os.path.join(b.ROCM, "include")]
if src == "bindings.cpp":
    cmd += ["-DTORCH_EXTENSION_NAME=_C"] + sum((["-I", p] for p in tinc), []) + ["-I", sysconfig.get_paths()["include"]]
subprocess.run(cmd + ["-c", f"build/ab/{src}", "-o", f"build/ab/{src}.o"], check=True)
PY
    ;;
  esac
  objs=$(echo $objs | sed "s|build/obj/$src.o|build/ab/$src.o|")
done
# symbols the current bindings need that the old sources lack: weak no-op stubs (AB_STUBS="name ...")
if [ -n "$AB_STUBS" ]; then
  : > build/ab/stubs.c
  for f in $AB_STUBS; do echo "__attribute__((weak)) void $f(long x) { (void)x; }" >> build/ab/stubs.c; done
  gcc -c -fPIC build/ab/stubs.c -o build/ab/stubs.o
  objs="$objs build/ab/stubs.o"
fi
TL=$(python -c "import torch,os;print(os.path.join(os.path.dirname(torch.__file__),'lib'))")
g++ -shared -o ab/_C_base.so $objs -L$TL -L/opt/rocm/lib -Wl,-rpath,$TL -Wl,-rpath,/opt/rocm/lib -lc10 -lc10_hip -ltorch -ltorch_cpu -ltorch_hip -ltorch_python -lamdhip64 -lz
echo "built ab/_C_base.so from $rev: $*"
