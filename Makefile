# Build libqhuff.so (product: HIP kernels for gfx950 + C drop-ins) and the
# oracle's CPU library (test infrastructure).  Used by __graft_entry__.build().
HIPCC   ?= /opt/rocm/bin/hipcc
CC      ?= gcc
ARCH    ?= gfx950
CSRC    := nghttp3_amd/csrc
LIBDIR  := nghttp3_amd/lib
LIB     := $(LIBDIR)/libqhuff.so
ARCHIVE := $(LIBDIR)/libqhuff.a
ORACLE  := oracle/libqh_oracle.so

HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -fvisibility=hidden \
            -Wall -Wno-unused-function -Wno-unused-value -Wno-unused-result
CFLAGS   := -std=c11 -O2 -fPIC -fvisibility=hidden -Wall -Wextra

DRIVER  := $(LIBDIR)/qpack

all: $(LIB) $(ARCHIVE) $(DRIVER) $(ORACLE)

$(CSRC)/qh_tables.h: nghttp3_amd/tools/gen_tables.py
	python3 nghttp3_amd/tools/gen_tables.py $@

$(LIBDIR)/qh_scalar.o: $(CSRC)/qh_scalar.c $(CSRC)/qh_tables.h include/qhuff.h
	@mkdir -p $(LIBDIR)
	$(CC) $(CFLAGS) -c $< -o $@

$(LIBDIR)/qh_device.o: $(CSRC)/qh_device.hip $(CSRC)/*.inc $(CSRC)/qh_common.h $(CSRC)/qh_tables.h $(CSRC)/qh_tokens.h $(CSRC)/qh_qpack_core.h $(CSRC)/qh_frame_fast.h include/qhuff.h
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/qh_qpack.o: $(CSRC)/qh_qpack.c $(CSRC)/qh_qpack_core.h include/qhuff.h
	@mkdir -p $(LIBDIR)
	$(CC) $(CFLAGS) -c $< -o $@

$(LIBDIR)/qh_static.o: $(CSRC)/qh_static.c include/qhuff.h
	@mkdir -p $(LIBDIR)
	$(CC) $(CFLAGS) -c $< -o $@

$(LIBDIR)/qh_http.o: $(CSRC)/qh_http.c $(CSRC)/qh_tokens.h include/qhuff.h
	@mkdir -p $(LIBDIR)
	$(CC) $(CFLAGS) -c $< -o $@

$(LIB): $(LIBDIR)/qh_device.o $(LIBDIR)/qh_scalar.o $(LIBDIR)/qh_qpack.o $(LIBDIR)/qh_http.o $(LIBDIR)/qh_static.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^

# The QIF bench driver (examples/qpack.cc counterpart), linked against the
# shared library next to it.
$(DRIVER): $(CSRC)/qh_qif.cc include/qhuff.h $(LIB)
	$(CXX) -std=c++17 -O2 -Wall -Wextra -o $@ $< -L$(LIBDIR) -lqhuff \
	  -Wl,-rpath,'$$ORIGIN' -Wl,-rpath-link,/opt/rocm/lib

# Static archive of the same two objects, for linking into libnghttp3 in
# place of the reference's Huffman objects.
$(ARCHIVE): $(LIBDIR)/qh_device.o $(LIBDIR)/qh_scalar.o $(LIBDIR)/qh_qpack.o $(LIBDIR)/qh_http.o $(LIBDIR)/qh_static.o
	rm -f $@
	ar rcs $@ $^

# Phase-timer build for kernel development (not loaded unless QHUFF_LIB
# points at it).
STAMPS := $(LIBDIR)/libqhuff_stamps.so
stamps: $(STAMPS)
$(STAMPS): $(CSRC)/qh_device.hip $(CSRC)/*.inc dev/csrc/*.inc $(CSRC)/qh_common.h $(LIBDIR)/qh_scalar.o $(LIBDIR)/qh_qpack.o $(LIBDIR)/qh_http.o $(LIBDIR)/qh_static.o
	$(HIPCC) $(HIPFLAGS) -DQH_STAMPS -DQH_STEP_COUNTS=1 -c $< -o $(LIBDIR)/qh_device_stamps.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(LIBDIR)/qh_device_stamps.o $(LIBDIR)/qh_scalar.o $(LIBDIR)/qh_qpack.o $(LIBDIR)/qh_http.o $(LIBDIR)/qh_static.o

# Development build with every kernel variant, after
#   git apply dev/patches/dev_variants_api.patch
# (the variants' host side, kept out of the product API; -DQH_DEV_VARIANTS: decoders
# fsm / fsm2 / lut / run / other peek widths and queue shapes, the
# chunk-engine and streaming encoders), selected by QHUFF_DECODER /
# QHUFF_ENCODER / QHUFF_CODES; loaded only when QHUFF_LIB points at it
# (dev/scripts/dec_variants.py).
DEV := $(LIBDIR)/libqhuff_dev.so
dev: $(DEV)
$(DEV): $(CSRC)/qh_device.hip $(CSRC)/*.inc dev/csrc/*.inc $(CSRC)/qh_common.h $(LIBDIR)/qh_scalar.o $(LIBDIR)/qh_qpack.o $(LIBDIR)/qh_http.o $(LIBDIR)/qh_static.o
	$(HIPCC) $(HIPFLAGS) -DQH_DEV_VARIANTS -Idev/csrc -c $< -o $(LIBDIR)/qh_device_dev.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(LIBDIR)/qh_device_dev.o $(LIBDIR)/qh_scalar.o $(LIBDIR)/qh_qpack.o $(LIBDIR)/qh_http.o $(LIBDIR)/qh_static.o

# Oracle: -O2 -mavx2 as nghttp3's README.rst:61-67 prescribes for the
# reference build (the Huffman loop itself has no SIMD path).
$(ORACLE): oracle/qh_oracle.c oracle/qh_oracle.h
	$(CC) -std=c11 -O2 -mavx2 -fPIC -shared -pthread -Wall -o $@ $<

clean:
	rm -f $(LIBDIR)/*.o $(DRIVER) $(LIB) $(ARCHIVE) $(STAMPS) $(DEV) $(ORACLE)

.PHONY: all clean stamps

# Fused-encoder ablation builds (timing experiments; wrong bytes):
# make abl ABL=<mask> -> libqhuff_abl<mask>.so (qh_enc_fused.inc QH_EW_ABL)
ABL ?= 0
abl: $(LIBDIR)/libqhuff_abl$(ABL).so
$(LIBDIR)/libqhuff_abl$(ABL).so: $(CSRC)/qh_device.hip $(CSRC)/*.inc $(CSRC)/qh_common.h $(LIBDIR)/qh_scalar.o $(LIBDIR)/qh_qpack.o $(LIBDIR)/qh_http.o $(LIBDIR)/qh_static.o
	$(HIPCC) $(HIPFLAGS) -DQH_EW_ABL=$(ABL) -c $< -o $(LIBDIR)/qh_device_abl$(ABL).o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(LIBDIR)/qh_device_abl$(ABL).o $(LIBDIR)/qh_scalar.o $(LIBDIR)/qh_qpack.o $(LIBDIR)/qh_http.o $(LIBDIR)/qh_static.o

# Framing without the LDS stage (development timing: every block parsed from
# global memory at the occupancy registers allow) -> libqhuff_frns.so
frns: $(LIBDIR)/libqhuff_frns.so
$(LIBDIR)/libqhuff_frns.so: $(CSRC)/qh_device.hip $(CSRC)/*.inc $(CSRC)/qh_common.h $(LIBDIR)/qh_scalar.o $(LIBDIR)/qh_qpack.o $(LIBDIR)/qh_http.o $(LIBDIR)/qh_static.o
	$(HIPCC) $(HIPFLAGS) -DQH_FRAME_NO_STAGE -c $< -o $(LIBDIR)/qh_device_frns.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(LIBDIR)/qh_device_frns.o $(LIBDIR)/qh_scalar.o $(LIBDIR)/qh_qpack.o $(LIBDIR)/qh_http.o $(LIBDIR)/qh_static.o

# Count-pass ablations (development timing: make frx FRX=<mask>, see
# QH_FR_ABL in qh_frame.inc) -> libqhuff_frx<mask>.so
frx: $(LIBDIR)/libqhuff_frx$(FRX).so
$(LIBDIR)/libqhuff_frx$(FRX).so: $(CSRC)/qh_device.hip $(CSRC)/*.inc $(CSRC)/qh_common.h $(LIBDIR)/qh_scalar.o $(LIBDIR)/qh_qpack.o $(LIBDIR)/qh_http.o $(LIBDIR)/qh_static.o
	$(HIPCC) $(HIPFLAGS) -DQH_FR_ABL=$(FRX) -c $< -o $(LIBDIR)/qh_device_frx$(FRX).o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(LIBDIR)/qh_device_frx$(FRX).o $(LIBDIR)/qh_scalar.o $(LIBDIR)/qh_qpack.o $(LIBDIR)/qh_http.o $(LIBDIR)/qh_static.o

# Length-pass ablations (development timing: make lx LX=<mask>, see
# QH_LX_ABL in qh_lane_enc.inc) -> libqhuff_lx<mask>.so
lx: $(LIBDIR)/libqhuff_lx$(LX).so
$(LIBDIR)/libqhuff_lx$(LX).so: $(CSRC)/qh_device.hip $(CSRC)/*.inc $(CSRC)/qh_common.h $(LIBDIR)/qh_scalar.o $(LIBDIR)/qh_qpack.o $(LIBDIR)/qh_http.o $(LIBDIR)/qh_static.o
	$(HIPCC) $(HIPFLAGS) -DQH_LX_ABL=$(LX) -c $< -o $(LIBDIR)/qh_device_lx$(LX).o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(LIBDIR)/qh_device_lx$(LX).o $(LIBDIR)/qh_scalar.o $(LIBDIR)/qh_qpack.o $(LIBDIR)/qh_http.o $(LIBDIR)/qh_static.o

# Codes-pass ablations (development timing: make la LA=<mask>, see QH_LA_ABL
# in qh_lane_enc.inc) -> libqhuff_la<mask>.so
la: $(LIBDIR)/libqhuff_la$(LA).so
$(LIBDIR)/libqhuff_la$(LA).so: $(CSRC)/qh_device.hip $(CSRC)/*.inc $(CSRC)/qh_common.h $(LIBDIR)/qh_scalar.o $(LIBDIR)/qh_qpack.o $(LIBDIR)/qh_http.o $(LIBDIR)/qh_static.o
	$(HIPCC) $(HIPFLAGS) -DQH_LA_ABL=$(LA) -c $< -o $(LIBDIR)/qh_device_la$(LA).o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(LIBDIR)/qh_device_la$(LA).o $(LIBDIR)/qh_scalar.o $(LIBDIR)/qh_qpack.o $(LIBDIR)/qh_http.o $(LIBDIR)/qh_static.o

# Dense-pack ablations (development timing: make dp DP=<mask>, see QH_DP_ABL
# in qh_host.inc) -> libqhuff_dp<mask>.so
dp: $(LIBDIR)/libqhuff_dp$(DP).so
$(LIBDIR)/libqhuff_dp$(DP).so: $(CSRC)/qh_device.hip $(CSRC)/*.inc $(CSRC)/qh_common.h $(LIBDIR)/qh_scalar.o $(LIBDIR)/qh_qpack.o $(LIBDIR)/qh_http.o $(LIBDIR)/qh_static.o
	$(HIPCC) $(HIPFLAGS) -DQH_DP_ABL=$(DP) -c $< -o $(LIBDIR)/qh_device_dp$(DP).o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(LIBDIR)/qh_device_dp$(DP).o $(LIBDIR)/qh_scalar.o $(LIBDIR)/qh_qpack.o $(LIBDIR)/qh_http.o $(LIBDIR)/qh_static.o

# Phase timers without step counts (development: framing phases, dev/scripts/frame_stamps.py)
frst: $(LIBDIR)/libqhuff_frst.so
$(LIBDIR)/libqhuff_frst.so: $(CSRC)/qh_device.hip $(CSRC)/*.inc $(CSRC)/qh_common.h $(LIBDIR)/qh_scalar.o $(LIBDIR)/qh_qpack.o $(LIBDIR)/qh_http.o $(LIBDIR)/qh_static.o
	$(HIPCC) $(HIPFLAGS) -DQH_STAMPS -c $< -o $(LIBDIR)/qh_device_frst.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(LIBDIR)/qh_device_frst.o $(LIBDIR)/qh_scalar.o $(LIBDIR)/qh_qpack.o $(LIBDIR)/qh_http.o $(LIBDIR)/qh_static.o

# The fused encoder at its free register allocation (3 waves per SIMD), for
# timing against the product's 4 -> libqhuff_ew3.so
ew3: $(LIBDIR)/libqhuff_ew3.so
$(LIBDIR)/libqhuff_ew3.so: $(CSRC)/qh_device.hip $(CSRC)/*.inc $(CSRC)/qh_common.h $(LIBDIR)/qh_scalar.o $(LIBDIR)/qh_qpack.o $(LIBDIR)/qh_http.o $(LIBDIR)/qh_static.o
	$(HIPCC) $(HIPFLAGS) -DQH_EW_MIN_WAVES=0 -c $< -o $(LIBDIR)/qh_device_ew3.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(LIBDIR)/qh_device_ew3.o $(LIBDIR)/qh_scalar.o $(LIBDIR)/qh_qpack.o $(LIBDIR)/qh_http.o $(LIBDIR)/qh_static.o

# Framing count pass with FRC blocks per wave (development timing:
# make frc FRC=16|32) -> libqhuff_frc<FRC>.so
frc: $(LIBDIR)/libqhuff_frc$(FRC).so
$(LIBDIR)/libqhuff_frc$(FRC).so: $(CSRC)/qh_device.hip $(CSRC)/*.inc $(CSRC)/qh_common.h $(LIBDIR)/qh_scalar.o $(LIBDIR)/qh_qpack.o $(LIBDIR)/qh_http.o $(LIBDIR)/qh_static.o
	$(HIPCC) $(HIPFLAGS) -DQH_FR_COUNT=$(FRC) -c $< -o $(LIBDIR)/qh_device_frc$(FRC).o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(LIBDIR)/qh_device_frc$(FRC).o $(LIBDIR)/qh_scalar.o $(LIBDIR)/qh_qpack.o $(LIBDIR)/qh_http.o $(LIBDIR)/qh_static.o

# Codes-pass occupancy variants (development timing: make encw5 EW=<waves>
# ES=<stage bytes>) -> libqhuff_ew<EW>s<ES>.so
encw5: $(LIBDIR)/libqhuff_ew$(EW)s$(ES).so
$(LIBDIR)/libqhuff_ew$(EW)s$(ES).so: $(CSRC)/qh_device.hip $(CSRC)/*.inc $(CSRC)/qh_common.h $(LIBDIR)/qh_scalar.o $(LIBDIR)/qh_qpack.o $(LIBDIR)/qh_http.o $(LIBDIR)/qh_static.o
	$(HIPCC) $(HIPFLAGS) -DQH_ENC_WAVES=$(EW) -DQH_ENC_STAGE=$(ES) -c $< -o $(LIBDIR)/qh_device_ew$(EW)s$(ES).o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(LIBDIR)/qh_device_ew$(EW)s$(ES).o $(LIBDIR)/qh_scalar.o $(LIBDIR)/qh_qpack.o $(LIBDIR)/qh_http.o $(LIBDIR)/qh_static.o

# a build with extra defines: make var V=<name> D="-DQH_...=..."
var: $(LIBDIR)/libqhuff_v$(V).so
$(LIBDIR)/libqhuff_v$(V).so: $(CSRC)/qh_device.hip $(CSRC)/*.inc $(CSRC)/qh_common.h $(LIBDIR)/qh_scalar.o $(LIBDIR)/qh_qpack.o $(LIBDIR)/qh_http.o $(LIBDIR)/qh_static.o
	$(HIPCC) $(HIPFLAGS) $(D) -c $< -o $(LIBDIR)/qh_device_v$(V).o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(LIBDIR)/qh_device_v$(V).o $(LIBDIR)/qh_scalar.o $(LIBDIR)/qh_qpack.o $(LIBDIR)/qh_http.o $(LIBDIR)/qh_static.o
