# Build of the MI355X raycaster (gfx950) — everything in-tree.
#
#   make            libraycast_hip.so (HIP kernels + C-ABI), libraycast_front.so (host
#                   scene parser / P3 writer), bin/raytrace (drop-in CLI), oracle
#   make ref        oracle/_ref: the reference C/ sources compiled in place (test oracle)
#
# Numerics flags (parity with the x86-64 gcc -O3 reference):
#   -ffp-contract=off                    no a*b+c fusion (hipcc defaults to fast-honor-pragmas)
#   -fno-gpu-flush-denormals-to-zero     f32 denormals kept, like SSE2
#   -fhip-fp32-correctly-rounded-divide-sqrt   IEEE f32 division
# Host C: gcc -O3 without -march (no FMA), like C/Makefile:4.

HIPCC   ?= /opt/rocm/bin/hipcc
CC      ?= gcc
PKG     := raytracing-programs_amd
SRC     := $(PKG)/csrc
LIB     := $(PKG)/lib
BIN     := $(PKG)/bin
OBJ     := $(PKG)/lib/obj
ARCH    ?= gfx950

HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off \
            -fno-gpu-flush-denormals-to-zero -fhip-fp32-correctly-rounded-divide-sqrt \
            -Iinclude -I$(SRC) -Wall -Wno-gnu-anonymous-struct -Wno-nested-anon-types \
            -Wno-c11-extensions -Wno-unused-result
CFLAGS   := -O3 -ffp-contract=off -fPIC -Wall -Wno-unused-result -Iinclude -I$(SRC)

HIP_SRCS  := $(SRC)/rc_kernels.hip $(SRC)/rc_api.hip $(SRC)/rc_shard.hip
HIP_HDRS  := $(SRC)/rc_device.hpp $(SRC)/rc_cudasem.hpp $(SRC)/rc_kernels.h $(SRC)/rc_runtime.h $(SRC)/rc_scene.h include/raycast_hip.h
FRONT_SRC := $(SRC)/front/parse.c $(SRC)/front/objects.c $(SRC)/front/ppm.c

.PHONY: all oracle ref clean stamps stamps2 sanitize
all: $(LIB)/libraycast_hip.so $(LIB)/libraycast_front.so $(BIN)/raytrace oracle

$(OBJ)/%.o: $(SRC)/%.hip $(HIP_HDRS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJ)/rc_scene.o: $(SRC)/rc_scene.c $(SRC)/rc_scene.h include/raycast_hip.h
	@mkdir -p $(OBJ)
	$(CC) $(CFLAGS) -c $< -o $@

ROCM    ?= /opt/rocm
HIPLIBS := -L$(ROCM)/lib -lrccl -Wl,-rpath,$(ROCM)/lib -lpthread

$(LIB)/libraycast_hip.so: $(OBJ)/rc_kernels.o $(OBJ)/rc_api.o $(OBJ)/rc_shard.o $(OBJ)/rc_scene.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $^ -o $@ $(HIPLIBS)

$(LIB)/libraycast_front.so: $(FRONT_SRC) include/raycast_hip.h
	@mkdir -p $(LIB)
	$(CC) $(CFLAGS) -shared $(FRONT_SRC) -o $@ -lm -lpthread

$(BIN)/raytrace: $(SRC)/front/raytrace_main.c $(LIB)/libraycast_front.so $(LIB)/libraycast_hip.so
	@mkdir -p $(BIN)
	$(CC) $(CFLAGS) $< -L$(LIB) -lraycast_front -lraycast_hip -Wl,-rpath,'$$ORIGIN/../lib' -o $@

# diagnostic build with in-kernel cycle stamps and the RC_RESOLVE_TRACE / RC_SIDE_STATS dumps
# (RC_HIP_LIB=libraycast_hip_stamps.so); the product library reads only RAYCAST_* options
stamps: $(LIB)/libraycast_hip_stamps.so
$(OBJ)/stamps_kernels.o: $(SRC)/rc_kernels.hip $(HIP_HDRS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -DRC_STAMPS=1 -DRC_DIAG=1 -c $< -o $@
$(OBJ)/stamps_api.o: $(SRC)/rc_api.hip $(HIP_HDRS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -DRC_STAMPS=1 -DRC_DIAG=1 -c $< -o $@
$(LIB)/libraycast_hip_stamps.so: $(OBJ)/stamps_kernels.o $(OBJ)/stamps_api.o $(OBJ)/rc_shard.o $(OBJ)/rc_scene.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $^ -o $@ $(HIPLIBS)
# coarse stamps: only per-step cycle counts (the evaluator itself is the product code)
stamps2: $(LIB)/libraycast_hip_stamps2.so
$(OBJ)/stamps2_kernels.o: $(SRC)/rc_kernels.hip $(HIP_HDRS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -DRC_STAMPS=2 -DRC_DIAG=1 -c $< -o $@
$(OBJ)/stamps2_api.o: $(SRC)/rc_api.hip $(HIP_HDRS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -DRC_STAMPS=2 -DRC_DIAG=1 -c $< -o $@
$(LIB)/libraycast_hip_stamps2.so: $(OBJ)/stamps2_kernels.o $(OBJ)/stamps2_api.o $(OBJ)/rc_shard.o $(OBJ)/rc_scene.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $^ -o $@ $(HIPLIBS)

oracle:
	$(MAKE) -C oracle oracle

ref:
	$(MAKE) -C oracle ref

clean:
	rm -rf $(LIB) $(BIN)
	$(MAKE) -C oracle clean

# measurement variants of the pixel kernels' framebuffer store (RC_HIP_LIB=libraycast_hip_<v>.so):
#   coalesced: 32x8 tiles staged in LDS, whole-row stores; t16: 16x16 tiles staged in LDS
variants: $(LIB)/libraycast_hip_coalesced.so $(LIB)/libraycast_hip_t16.so
$(OBJ)/coalesced_kernels.o: $(SRC)/rc_kernels.hip $(HIP_HDRS)
	$(HIPCC) $(HIPFLAGS) -DRC_TILE_W=32 -DRC_TILE_STAGE=1 -c $< -o $@
$(OBJ)/t16_kernels.o: $(SRC)/rc_kernels.hip $(HIP_HDRS)
	$(HIPCC) $(HIPFLAGS) -DRC_TILE_W=16 -DRC_TILE_STAGE=1 -c $< -o $@
# occupancy variants of the pixel kernels (RC_PHASE_A_WAVES waves per SIMD)
$(OBJ)/pa5_kernels.o: $(SRC)/rc_kernels.hip $(HIP_HDRS)
	$(HIPCC) $(HIPFLAGS) -DRC_PHASE_A_WAVES=5 -c $< -o $@
$(OBJ)/pa6_kernels.o: $(SRC)/rc_kernels.hip $(HIP_HDRS)
	$(HIPCC) $(HIPFLAGS) -DRC_PHASE_A_WAVES=6 -c $< -o $@
$(LIB)/libraycast_hip_%.so: $(OBJ)/%_kernels.o $(OBJ)/rc_api.o $(OBJ)/rc_shard.o $(OBJ)/rc_scene.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $^ -o $@ $(HIPLIBS)

# ASan + UBSan builds of the host C (tests/test_sanitize.py; SURVEY.md §5: the CPU restatement
# must not rely on UB): the oracle's CLI and the front end (parse / lists / P3 writer) driven
# by tests/tools/front_check.c.  Host code only; no GPU code is sanitized.
SAN     := -fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g
SAN_OUT := build/sanitize
sanitize: $(SAN_OUT)/oracle_raytrace $(SAN_OUT)/front_check
$(SAN_OUT)/oracle_raytrace: oracle/oracle_main.c oracle/rc_oracle.c oracle/rc_oracle.h include/raycast_hip.h
	@mkdir -p $(SAN_OUT)
	$(CC) -O1 -ffp-contract=off $(SAN) -Iinclude oracle/oracle_main.c oracle/rc_oracle.c -o $@ -lm
$(SAN_OUT)/front_check: tests/tools/front_check.c $(FRONT_SRC) include/raycast_hip.h
	@mkdir -p $(SAN_OUT)
	$(CC) -O1 -ffp-contract=off $(SAN) -Iinclude -I$(SRC) tests/tools/front_check.c $(FRONT_SRC) -o $@ -lm -lpthread

# occupancy variants of the pixel kernels (RC_HIP_LIB=libraycast_hip_<v>.so): w3 = phase A /
# k_render compiled for 3 waves per SIMD (no VGPR spills), f3 = phase C (k_dep_chunks, k_finish)
occupancy: $(LIB)/libraycast_hip_w3.so $(LIB)/libraycast_hip_f3.so $(LIB)/libraycast_hip_c512.so $(LIB)/libraycast_hip_c2048.so
$(OBJ)/c512_kernels.o: $(SRC)/rc_kernels.hip $(HIP_HDRS)
	$(HIPCC) $(HIPFLAGS) -DRC_CHUNK=512 -c $< -o $@
$(OBJ)/c2048_kernels.o: $(SRC)/rc_kernels.hip $(HIP_HDRS)
	$(HIPCC) $(HIPFLAGS) -DRC_CHUNK=2048 -c $< -o $@
$(OBJ)/w3_kernels.o: $(SRC)/rc_kernels.hip $(HIP_HDRS)
	$(HIPCC) $(HIPFLAGS) -DRC_PHASE_A_WAVES=3 -c $< -o $@
$(OBJ)/f3_kernels.o: $(SRC)/rc_kernels.hip $(HIP_HDRS)
	$(HIPCC) $(HIPFLAGS) -DRC_FINISH_WAVES=3 -c $< -o $@
