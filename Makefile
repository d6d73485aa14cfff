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
OBJS := $(BUILD)/trace.o $(BUILD)/render.o $(BUILD)/bvh.o $(BUILD)/ploc.o $(BUILD)/split.o $(BUILD)/bvh8.o $(BUILD)/path.o $(BUILD)/subtree.o $(BUILD)/context.o $(BUILD)/objloader.o

all: $(LIBDIR)/libpgrt.so $(LIBDIR)/libpgrt_image.so oracle $(BUILD)/pg1_pgrt

$(BUILD) $(LIBDIR):
	mkdir -p $@

HDRS := include/pgrt.h include/pgrt_detmath.h $(SRC)/cache_ops.hpp $(SRC)/stamps.hpp $(SRC)/common.hpp $(SRC)/trace.hpp $(SRC)/traverse.hpp $(SRC)/shade_ops.hpp $(SRC)/camera_ops.hpp $(SRC)/shade_ray.hpp $(SRC)/tiles.hpp $(SRC)/path.hpp

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

clean:
	rm -rf $(BUILD) $(LIBDIR)/libpgrt.so
	$(MAKE) -C oracle clean

.PHONY: all oracle clean
