# Top-level build: the product library (HIP, gfx950) and the CPU oracle (test infrastructure).
#   make            -> voxelraytracer_amd/_lib/libvrt.so + oracle/build/liboracle.so
# Numerics flags are part of the parity contract (DESIGN.md "Numerics"): no FP contraction,
# correctly rounded f32 div/sqrt on the device.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
LIBDIR := voxelraytracer_amd/_lib
# -fno-slp-vectorize: packed-FP32 (v_pk_*) ops take two issue slots on gfx950, no gain here
HIPFLAGS := -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -ffp-contract=off \
            -fhip-fp32-correctly-rounded-divide-sqrt -fno-slp-vectorize -Iinclude -Wall
SRC := voxelraytracer_amd/csrc/vrt_render.hip voxelraytracer_amd/csrc/vrt_context.cpp \
       voxelraytracer_amd/csrc/vrt_host.cpp
HDR := include/vrt.h voxelraytracer_amd/csrc/vrt_internal.h
# RCCL: volume broadcast and the frame gather of multi-device contexts (vrt_context.cpp)
LIBS := -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

all: $(LIBDIR)/libvrt.so oracle app

$(LIBDIR)/libvrt.so: $(SRC) $(HDR)
	mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(SRC) $(LIBS)

oracle:
	$(MAKE) -C oracle

# headless C++ host of the frame loop (examples/headless_app.cpp), linked against the C-ABI
app: build/bin/vrt_headless

build/bin/vrt_headless: examples/headless_app.cpp $(HDR) $(LIBDIR)/libvrt.so
	mkdir -p build/bin
	g++ -O2 -std=c++17 -Wall -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ -o $@ \
	    examples/headless_app.cpp -L$(LIBDIR) -lvrt -L/opt/rocm/lib -lamdhip64 \
	    -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)' -Wl,-rpath,/opt/rocm/lib

# experiment / diagnostic variants for scripts/ab.py, stamps.py, cert_diag.py (never the product
# library): make variant NAME=w6 DEFS="-DVRT_MIN_WAVES=6", NAME=stamps DEFS=-DVRT_STAMPS
variant: $(SRC) $(HDR)
	mkdir -p build/variants
	$(HIPCC) $(HIPFLAGS) -DVRT_DIAGNOSTIC_BUILD $(DEFS) -shared -o build/variants/libvrt_$(NAME).so $(SRC) $(LIBS)

asm: $(SRC) $(HDR)
	mkdir -p build/asm
	$(HIPCC) $(HIPFLAGS) -c --cuda-device-only -S -o build/asm/vrt_render.s voxelraytracer_amd/csrc/vrt_render.hip
	$(HIPCC) $(HIPFLAGS) -c --cuda-device-only -Rpass-analysis=kernel-resource-usage -o /dev/null voxelraytracer_amd/csrc/vrt_render.hip

clean:
	rm -rf $(LIBDIR) build
	$(MAKE) -C oracle clean

.PHONY: all oracle app asm clean variant
