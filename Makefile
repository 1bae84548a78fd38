# Builds the MI355X (gfx950) library in-tree: usnetd_amd/libusn.so
# and the CPU oracle (test infrastructure) oracle/build/liboracle.so.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function
CSRC := usnetd_amd/csrc
LIB := usnetd_amd/libusn.so
OBJS := build/usn_device.o build/usn_device512.o build/usn_host.o

DAEMON := usnetd_amd/bin/usnetd

TESTLIB := build/test/libusn.so

all: $(LIB) $(TESTLIB) $(DAEMON) oracle

# the daemon: plain C++ over the C ABI (links libusn.so; no HIP code of its own)
$(DAEMON): usnetd_amd/daemon/usnetd.cpp usnetd_amd/daemon/messages.hpp usnetd_amd/daemon/json.hpp include/usn_classify.h $(LIB)
	@mkdir -p usnetd_amd/bin
	g++ -O2 -std=c++17 -Wall -Wextra -o $@ $< -Lusnetd_amd -lusn -Wl,-rpath,'$$ORIGIN/..' \
	    -Wl,-rpath-link,/opt/rocm/lib -lpthread

build/usn_device.o: $(CSRC)/usn_device.hip $(CSRC)/usn_internal.h $(CSRC)/usn_kernels.h include/usn_classify.h
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

build/usn_device512.o: $(CSRC)/usn_device.hip $(CSRC)/usn_internal.h $(CSRC)/usn_kernels.h include/usn_classify.h
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -DUSN_NTHREADS=512 -DUSN_NS=usn_t512 -c -o $@ $<

build/usn_host.o: $(CSRC)/usn_host.cpp $(CSRC)/usn_internal.h $(CSRC)/usn_kernels.h include/usn_classify.h
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -x hip -c -o $@ $<

$(LIB): $(OBJS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(OBJS)

# the test build: the product's device code with a host object that reads the
# A/B and test knobs of the environment (USN_TEST_HOOKS, usn_host.cpp).  Only
# tests that force failures and tools/abl.py's variants load it.
build/test/usn_host.o: $(CSRC)/usn_host.cpp $(CSRC)/usn_internal.h $(CSRC)/usn_kernels.h include/usn_classify.h
	@mkdir -p build/test
	$(HIPCC) $(HIPFLAGS) -DUSN_TEST_HOOKS=1 -x hip -c -o $@ $<

$(TESTLIB): build/usn_device.o build/usn_device512.o build/test/usn_host.o
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $^

oracle:
	$(MAKE) -s -C oracle

# kernel resource usage (VGPR/SGPR/LDS/occupancy) for DESIGN.md
resources: $(CSRC)/usn_device.hip
	$(HIPCC) $(HIPFLAGS) -c -o /dev/null $< -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E 'Function Name|VGPRs:|SGPRs:|Occupancy|LDS Size|ScratchSize'

asm: $(CSRC)/usn_device.hip
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -S --offload-device-only -o build/usn_device.s $<

clean:
	rm -rf build $(LIB) $(DAEMON)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean resources asm

# A/B experiment builds (tools/abl.py): build/abl/<variant>/libusn.so,
# one variant per line of tools/abl_variants.txt: "<name> <extra hipcc flags>"
# (USN_AB_BUILD=1: the A/B-only knobs that give wrong results are allowed
# here and nowhere else, usn_device.hip)
# (ABL_ONLY="v1 v2": only those)
abl: build/test/usn_host.o
	@while read -r name flags; do \
	  case "$$name" in ''|'#'*) continue;; esac; \
	  case " $(ABL_ONLY) " in "  ") ;; *" $$name "*) ;; *) continue;; esac; \
	  mkdir -p build/abl/$$name; echo "variant $$name: $$flags"; \
	  $(HIPCC) $(HIPFLAGS) -DUSN_AB_BUILD=1 $$flags -c -o build/abl/$$name/dev.o $(CSRC)/usn_device.hip & \
	  $(HIPCC) $(HIPFLAGS) -DUSN_AB_BUILD=1 -DUSN_NTHREADS=512 -DUSN_NS=usn_t512 $$flags -c -o build/abl/$$name/dev512.o $(CSRC)/usn_device.hip & \
	  wait; \
	  $(HIPCC) $(HIPFLAGS) -shared -o build/abl/$$name/libusn.so build/abl/$$name/dev.o build/abl/$$name/dev512.o build/test/usn_host.o || exit 1; \
	done < tools/abl_variants.txt
.PHONY: abl
