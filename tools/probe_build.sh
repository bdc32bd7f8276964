#!/bin/bash
# Probe builds: SRC.hip (default gemm_big, the window GEMM; also sensor, the cooperative CNN1D)
# compiled with -DF3_PROBE=N (see the file's header): fall_multimodal_amd/libfall3_probeN.so for
# each N given (default 1 2 4), the rest of the library as built by make. Time them with
# F3_LIB=... python tools/kbench.py KEYS (or tools/cnn1d_time.py).
set -e
cd "$(dirname "$0")/.."
make -s -j8
SRC=${SRC:-gemm_big}
OBJS=$(ls build/*.o | grep -v "/$SRC.o")
for N in ${@:-1 2 4}; do
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -Iinclude -Ifall_multimodal_amd/csrc -Wno-unused-result \
    -DF3_PROBE=$N -c fall_multimodal_amd/csrc/$SRC.hip -o build/probe/${SRC}_$N.o 2>/dev/null || \
    { mkdir -p build/probe && /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -Iinclude \
      -Ifall_multimodal_amd/csrc -Wno-unused-result -DF3_PROBE=$N -c fall_multimodal_amd/csrc/$SRC.hip \
      -o build/probe/${SRC}_$N.o; }
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o fall_multimodal_amd/libfall3_probe$N.so $OBJS \
    build/probe/${SRC}_$N.o
done
