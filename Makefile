# Build libpech_crc32c.so (gfx950 HIP kernels + C-ABI) in-tree, and the
# test-only oracle libraries.  `make` is what __graft_entry__.build() runs.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 --offload-arch=$(ARCH) -fPIC -Wall -Wno-unused-function
SRC = pech_amd/csrc/crc32c_kernels.hip pech_amd/csrc/crc32c_api.cpp pech_amd/csrc/crc32c_async.cpp \
      pech_amd/csrc/crc32c_cpu.c pech_amd/csrc/crc32c_msgr.c
CFLAGS_HOST ?= -O2 -std=gnu11 -fPIC -Wall -Wextra -Werror
HDR = pech_amd/csrc/gf2.h pech_amd/csrc/layout.h pech_amd/csrc/api_internal.h include/crc32c.h include/pech_crc32c.h \
      include/pech_crc32c_async.h include/pech_crc32c_msgr.h
LIB = pech_amd/libpech_crc32c.so
HOST_OBJ = build/crc32c_api.o build/crc32c_async.o build/crc32c_cpu.o build/crc32c_msgr.o
OBJ = build/crc32c_kernels.o $(HOST_OBJ)

# the reference sources exist in the build container only (never on the GPU box)
REF_PRESENT := $(wildcard /root/reference/src/ceph/messenger.c)

all: $(LIB) oracle build/msgr_sim build/msgr_conn_sim build/dropin_kat build/coro_stack build/dropin_bench build/launch_cost \
     build/lib_dbg.so build/lib_test.so build/hbm_probe build/sched_probe build/host_probe $(if $(REF_PRESENT),build/msgr_loopback)

build/crc32c_kernels.o: pech_amd/csrc/crc32c_kernels.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

build/crc32c_api.o: pech_amd/csrc/crc32c_api.cpp $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

build/crc32c_async.o: pech_amd/csrc/crc32c_async.cpp $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

# host routine + library stack: plain C, no HIP (never includes oracle/)
build/crc32c_cpu.o: pech_amd/csrc/crc32c_cpu.c pech_amd/csrc/gf2.h
	@mkdir -p build
	gcc $(CFLAGS_HOST) -c $< -o $@

build/crc32c_msgr.o: pech_amd/csrc/crc32c_msgr.c include/pech_crc32c_msgr.h include/pech_crc32c_async.h
	@mkdir -p build
	gcc $(CFLAGS_HOST) -c $< -o $@

$(LIB): $(OBJ)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(OBJ)

# device assembly for inspection (build/crc32c_kernels-hip-amdgcn-amd-amdhsa-gfx950.s)
asm: pech_amd/csrc/crc32c_kernels.hip $(HDR)
	@mkdir -p build
	cd build && $(HIPCC) $(HIPFLAGS) --cuda-device-only -S -Rpass-analysis=kernel-resource-usage \
		../pech_amd/csrc/crc32c_kernels.hip -o crc32c_kernels.s

# A/B diagnostic build: make variant V=name D="-DPECH_U=9" -> build/lib_name.so
variant: $(HOST_OBJ)
	$(HIPCC) $(HIPFLAGS) $(D) -c pech_amd/csrc/crc32c_kernels.hip -o build/k_$(V).o
	$(HIPCC) $(HIPFLAGS) -shared -o build/lib_$(V).so build/k_$(V).o $(HOST_OBJ)

# bounds-checked kernel build for the GPU test suite (tests/test_gpu_bounds.py):
# every ring load is checked against its buffer's core; a violation prints
# "PECH OOB" and is redirected instead of faulting
build/lib_dbg.so: pech_amd/csrc/crc32c_kernels.hip $(HDR) $(HOST_OBJ)
	$(HIPCC) $(HIPFLAGS) -DPECH_DEBUG_BOUNDS -c pech_amd/csrc/crc32c_kernels.hip -o build/k_dbg.o
	$(HIPCC) $(HIPFLAGS) -shared -o $@ build/k_dbg.o $(HOST_OBJ)

# test build for the failure-path tests (tests/test_faults.py): the same objects,
# except that crc32c_api is compiled with the fault-injection hook
# (crc32c_test_inject), which the release library does not have
build/crc32c_api_test.o: pech_amd/csrc/crc32c_api.cpp $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -DPECH_TEST_HOOKS -x hip -c $< -o $@

build/crc32c_async_test.o: pech_amd/csrc/crc32c_async.cpp $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -DPECH_TEST_HOOKS -x hip -c $< -o $@

build/lib_test.so: build/crc32c_kernels.o build/crc32c_api_test.o build/crc32c_async_test.o build/crc32c_cpu.o \
		   build/crc32c_msgr.o
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $^

# test program: pech's receive path on the async layer (gnu89, epoll loop);
# links the test oracle for the expected footer CRCs -- not product code
build/msgr_sim: tests/c/msgr_sim.c oracle/crc32c_oracle.c include/pech_crc32c_async.h $(LIB)
	@mkdir -p build
	gcc -std=gnu89 -O2 -Wall -Werror -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ \
		tests/c/msgr_sim.c oracle/crc32c_oracle.c -Lpech_amd -lpech_crc32c -L/opt/rocm/lib -lamdhip64 \
		-Wl,-rpath,'$$ORIGIN/../pech_amd' -o $@

# test program: messenger connection state machine on the adapter (send, receive
# verify queue, faults and resends, REPOP fan-out, option gates)
build/msgr_conn_sim: tests/c/msgr_conn_sim.c oracle/crc32c_oracle.c include/pech_crc32c_msgr.h $(LIB)
	@mkdir -p build
	gcc -std=gnu89 -O2 -Wall -Werror -Iinclude tests/c/msgr_conn_sim.c oracle/crc32c_oracle.c -Lpech_amd \
		-lpech_crc32c -Wl,-rpath,'$$ORIGIN/../pech_amd' -o $@

# test program (built in the build container, run on both sides): the
# reference messenger ITSELF, patched by integration/pech_crc32c_msgr.patch
# in a temp dir, linked with all of pech but main.c and with the library;
# tests/c/msgr_loopback.c is only its caller (tests/test_msgr_loopback.py)
build/msgr_loopback: tests/c/msgr_loopback.c tests/c/loopback_proxy.c tests/c/loopback_proxy.h tests/pech_build.py \
		     integration/pech_crc32c_msgr.patch oracle/crc32c_oracle.c include/pech_crc32c_msgr.h $(LIB)
	@mkdir -p build
	python3 tests/pech_build.py loopback $@

# test program: the drop-in crc32c() from C, as messenger.c calls it
build/dropin_kat: tests/c/dropin_kat.c include/crc32c.h $(LIB)
	@mkdir -p build
	gcc -std=gnu89 -O2 -Wall -Werror -Iinclude tests/c/dropin_kat.c -Lpech_amd -lpech_crc32c \
		-L/opt/rocm/lib -lamdhip64 -Wl,-rpath,'$$ORIGIN/../pech_amd' -o $@

# test program: the library from a 64 KiB pech-style coroutine stack
# (pech itself needs -D_FORTIFY_SOURCE=0 for its cross-stack longjmp)
build/coro_stack: tests/c/coro_stack.c oracle/crc32c_oracle.c include/pech_crc32c_async.h $(LIB)
	@mkdir -p build
	gcc -std=gnu89 -O2 -Wall -Werror -U_FORTIFY_SOURCE -D_FORTIFY_SOURCE=0 -Iinclude tests/c/coro_stack.c oracle/crc32c_oracle.c -Lpech_amd \
		-lpech_crc32c -Wl,-rpath,'$$ORIGIN/../pech_amd' -o $@

# bench tool: drop-in per-call latency, host vs GPU route vs the reference loop
build/dropin_bench: tools/c/dropin_bench.c oracle/crc32c_oracle.c include/pech_crc32c.h $(LIB)
	@mkdir -p build
	gcc -std=gnu89 -O2 -Wall -Werror -fno-strict-aliasing -Iinclude tools/c/dropin_bench.c oracle/crc32c_oracle.c \
		-Lpech_amd -lpech_crc32c -Wl,-rpath,'$$ORIGIN/../pech_amd' -o $@

# bench tool: host CPU per HIP call of an async-layer slot
build/launch_cost: tools/c/launch_cost.c include/pech_crc32c.h $(LIB)
	@mkdir -p build
	gcc -std=gnu89 -O2 -Wall -Werror -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ tools/c/launch_cost.c \
		-Lpech_amd -lpech_crc32c -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,'$$ORIGIN/../pech_amd' -o $@

oracle:
	$(MAKE) -C oracle all
	@if [ -d /root/reference/include ]; then $(MAKE) -C oracle ref; fi

clean:
	rm -rf build $(LIB)
	$(MAKE) -C oracle clean

.PHONY: all asm variant oracle clean

# GPU-box probes (not product code): HBM read shapes, work-distribution schedules
build/hbm_probe: tools/hbm_probe.hip
	@mkdir -p build
	$(HIPCC) -O3 --offload-arch=$(ARCH) $< -o $@

build/sched_probe: tools/sched_probe.hip
	@mkdir -p build
	$(HIPCC) -O3 --offload-arch=$(ARCH) $< -o $@

build/host_probe: tools/host_probe.hip
	@mkdir -p build
	$(HIPCC) -O3 --offload-arch=$(ARCH) $< -o $@
