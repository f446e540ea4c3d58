# Build of the MI355X UHSDR RX hot path (gfx950) and its CPU oracle.
#
#   make            -> uhsdr_amd/lib/libuhsdr_amd.so   (product: C-ABI, HIP kernels + host setup)
#                      oracle/build/libuhsdr_oracle.so (test infrastructure: CPU restatement)
#   make ref        -> oracle/_ref/uhsdr_ref           (reference firmware chain, needs /root/reference)
#
# Host C is compiled without FP contraction and without -march, like the reference build,
# so every binary32 rounding of the setup math and of the oracle matches the reference.

HIPCC   ?= /opt/rocm/bin/hipcc
CC      ?= gcc
ARCH    ?= gfx950
HOSTCFLAGS := -O2 -fPIC -ffp-contract=off -std=gnu11 -Wall -Wno-unused-function
HIPFLAGS   := --offload-arch=$(ARCH) -Iuhsdr_amd/csrc -O3 -fPIC -ffp-contract=off -fno-slp-vectorize -std=c++17 -Wno-unused-result

LIB     := uhsdr_amd/lib/libuhsdr_amd.so
CMSISLIB := uhsdr_amd/lib/libuhsdr_cmsis.so
ORACLE  := oracle/build/libuhsdr_oracle.so
OBJDIR  := uhsdr_amd/build

HOST_SRCS := uhsdr_amd/csrc/uhsdr_setup.c uhsdr_amd/csrc/uhsdr_filter_tables.c
HIP_SRCS  := uhsdr_amd/csrc/uhsdr_rx.hip uhsdr_amd/csrc/uhsdr_tx.hip uhsdr_amd/csrc/uhsdr_spectrum.hip uhsdr_amd/csrc/uhsdr_i2s.hip uhsdr_amd/csrc/uhsdr_fir.hip
HOST_OBJS := $(patsubst uhsdr_amd/csrc/%.c,$(OBJDIR)/%.o,$(HOST_SRCS))
HIP_OBJS  := $(patsubst uhsdr_amd/csrc/%.hip,$(OBJDIR)/%.o,$(HIP_SRCS))
HDRS := uhsdr_amd/csrc/uhsdr_rx_variants.inc include/uhsdr.h uhsdr_amd/csrc/uhsdr_internal.h uhsdr_amd/csrc/uhsdr_dsp.h uhsdr_amd/csrc/uhsdr_libm.h uhsdr_amd/csrc/uhsdr_cfft.h

EXAMPLE := examples/build/rx_batch

all: $(LIB) $(CMSISLIB) $(ORACLE) $(EXAMPLE)

$(OBJDIR) uhsdr_amd/lib oracle/build:
	mkdir -p $@

$(OBJDIR)/%.o: uhsdr_amd/csrc/%.c $(HDRS) | $(OBJDIR)
	$(CC) $(HOSTCFLAGS) -c $< -o $@

$(OBJDIR)/%.o: uhsdr_amd/csrc/%.hip $(HDRS) | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(HOST_OBJS) $(HIP_OBJS) | uhsdr_amd/lib
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $^ -lm

# CMSIS-DSP signature shims (include/uhsdr_cmsis.h): a library of their own, so the arm_* names
# never collide with a CMSIS build linked elsewhere; uses libuhsdr_amd.so's setup layer
$(OBJDIR)/uhsdr_cmsis.o: uhsdr_amd/csrc/uhsdr_cmsis.hip include/uhsdr_cmsis.h $(HDRS) | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CMSISLIB): $(OBJDIR)/uhsdr_cmsis.o $(LIB) | uhsdr_amd/lib
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(OBJDIR)/uhsdr_cmsis.o -Luhsdr_amd/lib -luhsdr_amd -Wl,-rpath,'$$ORIGIN' -lm

$(ORACLE): oracle/uhsdr_oracle.c oracle/uhsdr_oracle.h include/uhsdr.h | oracle/build
	$(CC) $(HOSTCFLAGS) -shared -o $@ $< -lm -lpthread

examples/build:
	mkdir -p $@

# plain C host against the C ABI: gcc only, no HIP headers
$(EXAMPLE): examples/rx_batch.c include/uhsdr.h $(LIB) | examples/build
	$(CC) -O2 -std=gnu11 -Wall -Iinclude -o $@ $< -Luhsdr_amd/lib -luhsdr_amd -Wl,-rpath,'$$ORIGIN/../../uhsdr_amd/lib'

ref:
	$(MAKE) -C oracle/ref

clean:
	rm -rf $(OBJDIR) uhsdr_amd/lib oracle/build examples/build

.PHONY: all ref clean

# compile-time variants of libuhsdr_amd.so for A/B measurement (bench.py with UHSDR_LIB=<path>):
#   make variant VTAG=w3 VFLAGS=-DUHSDR_FUSED_WAVES=3
# every HIP source is rebuilt with VFLAGS into its own object directory, so a flag read by any
# source takes effect (VFLAGS=-Itools/isa builds only the P48 receive kernels: quick A/B builds;
# VFLAGS comes first on the line, so its -I wins over csrc for uhsdr_rx_variants.inc)
VARIANT_DIR := uhsdr_amd/lib/variants
VOBJDIR = $(OBJDIR)/v_$(VTAG)
VHIP_OBJS = $(patsubst uhsdr_amd/csrc/%.hip,$(VOBJDIR)/%.o,$(HIP_SRCS))
$(OBJDIR)/v_%/.dir:
	mkdir -p $(dir $@) && touch $@
.PRECIOUS: $(OBJDIR)/v_%/.dir
$(VOBJDIR)/%.o: uhsdr_amd/csrc/%.hip $(HDRS) | $(VOBJDIR)/.dir
	$(HIPCC) $(VFLAGS) $(HIPFLAGS) -c $< -o $@
variant: $(HOST_OBJS) $(VHIP_OBJS)
	mkdir -p $(VARIANT_DIR)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $(VARIANT_DIR)/libuhsdr_amd_$(VTAG).so $(HOST_OBJS) $(VHIP_OBJS) -lm

.PHONY: variant
