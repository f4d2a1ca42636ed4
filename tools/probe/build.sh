#!/bin/bash
# Builds the launch probe: host binary + the kernel's code object for the AQL path.
set -e
cd "$(dirname "$0")"
/opt/rocm/bin/hipcc -O2 -std=c++17 --offload-arch=gfx950 launch_probe.hip -o launch_probe -lhsa-runtime64
/opt/rocm/bin/hipcc -O2 -std=c++17 --offload-arch=gfx950 --genco launch_probe.hip -o launch_probe.hsaco
/opt/rocm/llvm/bin/clang-offload-bundler --unbundle --type=o --input=launch_probe.hsaco \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=launch_probe.co
