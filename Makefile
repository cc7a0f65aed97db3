# Builds the product library udpdk_amd/libudpdk_amd.so (HIP kernels for gfx950 + C-ABI host code
# + the C udpdk_api.h host layer) and the test-only oracle (oracle/liboracle.so).
HIPCC     ?= /opt/rocm/bin/hipcc
CC        ?= gcc
ARCH      ?= gfx950
HIPFLAGS  ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Werror -Wno-unused-result
CFLAGS_H  ?= -O2 -std=gnu11 -fPIC -Wall -Wextra -Werror
INC       := -Iinclude -Iudpdk_amd/csrc
LIB       := udpdk_amd/libudpdk_amd.so
OBJDIR    := build/obj

HIP_SRC   := udpdk_amd/csrc/rx_kernels.hip udpdk_amd/csrc/rx_gather.hip udpdk_amd/csrc/rx_reasm.hip udpdk_amd/csrc/rx_rss.hip udpdk_amd/csrc/tx_kernels.hip \
             udpdk_amd/csrc/udpdk_gpu.hip
C_SRC     := $(wildcard udpdk_amd/csrc/host/*.c)
HIP_OBJ   := $(patsubst udpdk_amd/csrc/%.hip,$(OBJDIR)/%.o,$(HIP_SRC))
C_OBJ     := $(patsubst udpdk_amd/csrc/host/%.c,$(OBJDIR)/host/%.o,$(C_SRC))
HDRS      := include/udpdk_gpu.h include/udpdk_api.h udpdk_amd/csrc/rx_common.h \
             $(wildcard udpdk_amd/csrc/host/*.h)

TOOLS     := tools/bin/bench_sock

all: $(LIB) oracle $(TOOLS)

$(OBJDIR)/%.o: udpdk_amd/csrc/%.hip $(HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) $(INC) -c $< -o $@

$(OBJDIR)/host/%.o: udpdk_amd/csrc/host/%.c $(HDRS)
	@mkdir -p $(dir $@)
	$(CC) $(CFLAGS_H) $(INC) -c $< -o $@

$(LIB): $(HIP_OBJ) $(C_OBJ) udpdk_amd/csrc/libudpdk_amd.map
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $(HIP_OBJ) $(C_OBJ) -Wl,--no-undefined \
	    -Wl,-soname,libudpdk_amd.so -Wl,--version-script=udpdk_amd/csrc/libudpdk_amd.map

oracle: $(LIB)
	$(MAKE) -C oracle

# the reference-API path end to end, written against udpdk_api.h like a reference app (bench.py)
tools/bin/bench_sock: tools/bench_sock.c include/udpdk_api.h include/udpdk_gpu.h $(LIB)
	@mkdir -p tools/bin
	$(CC) -O2 -std=gnu11 -Wall -Wextra -Werror -Iinclude $< -o $@ -Ludpdk_amd -ludpdk_amd -Wl,-rpath,'$$ORIGIN/../../udpdk_amd'

# diagnostic library with per-phase s_memtime stamps (tools/stamps.py); never used by tests/bench
STAMP_LIB := tools/diag/libudpdk_amd.so
STAMP_OBJ := $(patsubst udpdk_amd/csrc/%.hip,build/stamps/%.o,$(HIP_SRC))
stamps: $(STAMP_LIB)
build/stamps/%.o: udpdk_amd/csrc/%.hip $(HDRS)
	@mkdir -p build/stamps
	$(HIPCC) $(HIPFLAGS) -DUDPDK_STAMPS $(INC) -c $< -o $@
$(STAMP_LIB): $(STAMP_OBJ) $(C_OBJ)
	@mkdir -p tools/diag
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $^ -Wl,--no-undefined

# diagnostic library with per-phase wall-clock timing inside udpdk_poll_rx (tools/sock_prof.sh)
PROF_LIB := tools/diag/pollprof/libudpdk_amd.so
PROF_OBJ := $(patsubst udpdk_amd/csrc/host/%.c,build/pollprof/%.o,$(C_SRC))
pollprof: $(PROF_LIB)
build/pollprof/%.o: udpdk_amd/csrc/host/%.c $(HDRS)
	@mkdir -p build/pollprof
	$(CC) $(CFLAGS_H) -DUDPDK_POLL_PROFILE $(INC) -c $< -o $@
$(PROF_LIB): $(HIP_OBJ) $(PROF_OBJ)
	@mkdir -p tools/diag/pollprof
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $^ -Wl,--no-undefined -Wl,-soname,libudpdk_amd.so

# A/B variant of the library (tools/ab.py): `make variant VAR=name VFLAGS="-DX=1"` builds
# tools/var/name.so from the same sources with extra compile flags; never used by tests/bench
VAR       ?= new
VFLAGS    ?=
VAR_OBJ   := $(patsubst udpdk_amd/csrc/%.hip,build/var/$(VAR)/%.o,$(HIP_SRC)) \
             $(patsubst udpdk_amd/csrc/host/%.c,build/var/$(VAR)/host/%.o,$(C_SRC))
variant: tools/var/$(VAR).so
build/var/$(VAR)/%.o: udpdk_amd/csrc/%.hip $(HDRS) FORCE
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) $(VFLAGS) $(INC) -c $< -o $@
build/var/$(VAR)/host/%.o: udpdk_amd/csrc/host/%.c $(HDRS) FORCE
	@mkdir -p $(dir $@)
	$(CC) $(CFLAGS_H) $(VFLAGS) $(INC) -c $< -o $@
tools/var/$(VAR).so: $(VAR_OBJ)
	@mkdir -p tools/var
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $^ -Wl,--no-undefined \
	    -Wl,-soname,libudpdk_amd.so -Wl,--version-script=udpdk_amd/csrc/libudpdk_amd.map
FORCE:

asm: udpdk_amd/csrc/rx_kernels.hip $(HDRS)
	@mkdir -p build/asm
	$(HIPCC) $(HIPFLAGS) -Wno-unused-command-line-argument $(INC) -S --cuda-device-only -o build/asm/rx_kernels.s $<
	$(HIPCC) $(HIPFLAGS) $(INC) -c -Rpass-analysis=kernel-resource-usage $< -o /dev/null 2> build/asm/rx_resource.txt || true

clean:
	rm -rf build $(LIB) $(TOOLS)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean asm stamps pollprof variant FORCE
