#!/bin/bash
# usage: mkvar.sh name "-DFLAGS..."
set -e
cd /root/repo
name=$1; flags=$2
mkdir -p build/var_$name tools/diag
for f in $(cd udpdk_amd/csrc && ls *.hip | sed "s/\.hip$//"); do hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $flags -Iinclude -Iudpdk_amd/csrc -c udpdk_amd/csrc/$f.hip -o build/var_$name/$f.o; done
hipcc -shared -fPIC --offload-arch=gfx950 -o tools/diag/lib_$name.so build/var_$name/*.o build/obj/host/*.o
