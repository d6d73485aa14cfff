# Build of libpgrt.so (gfx950 HIP kernels + C ABI) and the oracle (test infrastructure).
# Usage: make -j8            (driven by __graft_entry__.build())
HIPCC   ?= /opt/rocm/bin/hipcc
ARCH    ?= gfx950
BUILD   := build
LIBDIR  := pgi_raytracing_amd/lib
SRC     := pgi_raytracing_amd/csrc
# -ffp-contract=off: no implicit FMA, so every float op rounds exactly like the CPU restatement
HIPFLAGS := --offload-arch=$(ARCH) -O3 -fPIC -std=c++17 -ffp-contract=off \
            -fhip-fp32-correctly-rounded-divide-sqrt -Iinclude -I$(SRC) -Wall -Wno-unused-result
# shading kernels: no machine-level loop-invariant code motion -- it hoists the FP64 polynomial
# constants of the exact math (pgrt_detmath.h: exp / log / atan, no VOP3 literals on gfx9) out of
# the shading loop into SGPRs, which then spill (k_shade L0: 205 SGPR + 11 VGPR spills -> 73 + 0)
HIPFLAGS_render := -mllvm -disable-machine-licm
HIPFLAGS_path := -mllvm -disable-machine-licm
HIPFLAGS_trace := -mllvm -disable-machine-licm
HIPFLAGS_subtree := -mllvm -disable-machine-licm
OBJS := $(BUILD)/trace.o $(BUILD)/render.o $(BUILD)/bvh.o $(BUILD)/ploc.o $(BUILD)/split.o $(BUILD)/bvh8.o $(BUILD)/path.o \
        $(BUILD)/subtree.o $(BUILD)/context.o $(BUILD)/scene.o $(BUILD)/frame.o $(BUILD)/distributed.o \
        $(BUILD)/diagnostics.o $(BUILD)/tiles_abi.o $(BUILD)/objloader.o

all: $(LIBDIR)/libpgrt.so $(LIBDIR)/libpgrt_image.so oracle $(BUILD)/pg1_pgrt

$(BUILD) $(LIBDIR):
	mkdir -p $@

HDRS := include/pgrt.h include/pgrt_detmath.h $(SRC)/context.hpp $(SRC)/cache_ops.hpp $(SRC)/stamps.hpp $(SRC)/common.hpp $(SRC)/trace.hpp $(SRC)/traverse.hpp $(SRC)/shade_ops.hpp $(SRC)/camera_ops.hpp $(SRC)/shade_ray.hpp $(SRC)/tiles.hpp $(SRC)/path.hpp

$(BUILD)/%.o: $(SRC)/%.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) $(HIPFLAGS_$*) -c $< -o $@

$(BUILD)/%.o: $(SRC)/%.cpp $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/libpgrt.so: $(OBJS) | $(LIBDIR)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(OBJS) -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

# JPEG textures decoded like the reference's FreeImage JPEG_DEFAULT load (IJG libjpeg 9, IFAST
# IDCT, no fancy upsampling; csrc/image_jpeg.c).  libjpeg 9 ships with this image under /opt/conda.
JPEG_PREFIX ?= /opt/conda
# PNG through libpng 1.6 (also under /opt/conda), the format dispatch of Texture::Texture
$(LIBDIR)/libpgrt_image.so: $(SRC)/image_jpeg.c $(SRC)/image_png.c include/pgrt_image.h | $(LIBDIR)
	gcc -O2 -std=c11 -Wall -shared -fPIC -Iinclude -I$(JPEG_PREFIX)/include -o $@ $(SRC)/image_jpeg.c $(SRC)/image_png.c \
	    -L$(JPEG_PREFIX)/lib -ljpeg -lpng16 -Wl,-rpath,$(JPEG_PREFIX)/lib

# C++ host example over the C ABI (include/pgrt_raytracer.hpp)
$(BUILD)/pg1_pgrt: examples/pg1_pgrt.cpp include/pgrt_raytracer.hpp include/pgrt.h include/pgrt_image.h $(LIBDIR)/libpgrt.so $(LIBDIR)/libpgrt_image.so | $(BUILD)
	g++ -O2 -std=c++17 -Wall -Iinclude -o $@ $< -L$(LIBDIR) -lpgrt -lpgrt_image -Wl,-rpath,'$$ORIGIN/../$(LIBDIR)'

oracle:
	$(MAKE) -C oracle

# ---- host-side sanitizer build: `make asan`, then tools/asan_check.sh
# libpgrt.so whose HOST translation units (the C ABI, frame scheduling, distributed gather, OBJ
# loader, tile deal) are built with AddressSanitizer + UndefinedBehaviorSanitizer (clang's shared
# runtime; device code is the normal gfx950 build -- each -fsanitize applies to the host only),
# and the oracle (the CPU restatement) with the same sanitizers.  Outputs under build/asan/.
ASAN_DIR := $(BUILD)/asan
ASAN_HOST := -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=all \
             -Xarch_host -fno-omit-frame-pointer -shared-libasan -g
HOST_TUS := context scene frame distributed diagnostics tiles_abi objloader
ASAN_OBJS := $(patsubst %,$(ASAN_DIR)/%.o,$(HOST_TUS)) \
             $(filter-out $(patsubst %,$(BUILD)/%.o,$(HOST_TUS)),$(OBJS))
ORACLE_ASAN := /opt/rocm/lib/llvm/bin/clang -O1 -g -std=c11 -fPIC -ffp-contract=off -fno-fast-math -march=x86-64-v2 \
               -Wno-unknown-pragmas -Iinclude -fsanitize=address,undefined -fno-sanitize-recover=all \
               -fno-omit-frame-pointer -fno-gpu-sanitize -Wno-unused-command-line-argument -shared-libasan -shared

$(ASAN_DIR):
	mkdir -p $@

$(ASAN_DIR)/%.o: $(SRC)/%.cpp $(HDRS) | $(ASAN_DIR)
	$(HIPCC) $(HIPFLAGS) $(ASAN_HOST) -c $< -o $@

$(ASAN_DIR)/libpgrt.so: $(ASAN_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared $(ASAN_HOST) -o $@ $(ASAN_OBJS) -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

$(ASAN_DIR)/liboracle.so: oracle/oracle.c oracle/oracle.h include/pgrt.h include/pgrt_detmath.h | $(ASAN_DIR)
	$(ORACLE_ASAN) -o $@ oracle/oracle.c -lm

$(ASAN_DIR)/liboracle_libm.so: oracle/oracle.c oracle/oracle.h include/pgrt.h include/pgrt_detmath.h | $(ASAN_DIR)
	$(ORACLE_ASAN) -DORACLE_LIBM -o $@ oracle/oracle.c -lm

asan: $(ASAN_DIR)/libpgrt.so $(ASAN_DIR)/liboracle.so $(ASAN_DIR)/liboracle_libm.so

clean:
	rm -rf $(BUILD) $(LIBDIR)/libpgrt.so
	$(MAKE) -C oracle clean

.PHONY: all oracle clean asan
