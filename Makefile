# Top-level build: the HIP product library and the CPU parity oracle.
all: lib oracle ref abi

lib:
	$(MAKE) -C c_orb_slam_amd/csrc -j8

oracle:
	$(MAKE) -C oracle

# the reference's own libc-only sources (DUtils::Random) into oracle/_ref/, when /root/reference
# is present (this container); the GPU box uses the prebuilt oracle/_ref/ that travels with the tree
ref:
	if [ -f /root/reference/Thirdparty/DBoW2/DUtils/Random.cpp ]; then $(MAKE) -C oracle/ref; fi

# a plain C11 caller of include/orbslam_gpu.h linked against the product library
# (tests/test_library.py builds its own copy on CPU; the GPU test runs this one)
abi: build/abi_caller
build/abi_caller: tests/c_abi/abi_caller.c include/orbslam_gpu.h lib
	mkdir -p build
	gcc -std=c11 -pedantic -Wall -Wextra -Werror -O2 -Iinclude tests/c_abi/abi_caller.c \
	    -Lc_orb_slam_amd -lorbslam_gpu -Wl,-rpath,'$$ORIGIN/../c_orb_slam_amd' -o $@

clean:
	$(MAKE) -C c_orb_slam_amd/csrc clean
	$(MAKE) -C oracle clean

.PHONY: all lib oracle ref abi clean
