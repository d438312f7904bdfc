# Top-level build: the HIP product library and the CPU parity oracle.
all: lib oracle

lib:
	$(MAKE) -C c_orb_slam_amd/csrc -j8

oracle:
	$(MAKE) -C oracle

clean:
	$(MAKE) -C c_orb_slam_amd/csrc clean
	$(MAKE) -C oracle clean

.PHONY: all lib oracle clean
