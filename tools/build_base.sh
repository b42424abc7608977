#!/bin/bash
# Experiment helper: build libshdtopology_base.so from routes.hip at git revision $1 (default HEAD)
# next to the working-tree build, for A/B runs with SHDR_LIB_VARIANT=base.
set -e
cd "$(dirname "$0")/../shadow_amd"
rev=${1:-HEAD}
mkdir -p build_base
git show "$rev:shadow_amd/csrc/routes.hip" > csrc/routes_base_tmp.hip
trap 'rm -f csrc/routes_base_tmp.hip' EXIT
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -Wno-unused-parameter -c csrc/routes_base_tmp.hip -o build_base/routes.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o libshdtopology_base.so build/graph.o build/topology.o build/complete.o build/shim.o build_base/routes.o -pthread
