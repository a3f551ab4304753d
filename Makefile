# Top-level build: the product (libjmhip.so + host plumbing + lencod), the test-only oracle and the
# test harness binaries that combine the two (tests/harness).
.PHONY: all product oracle harness clean
all: product oracle harness

product:
	$(MAKE) -C h264-jm-commentary_amd/csrc libjmhip.so
	$(MAKE) -C h264-jm-commentary_amd/host all

oracle:
	$(MAKE) -C oracle all

harness: product oracle
	$(MAKE) -C tests/harness all

clean:
	$(MAKE) -C h264-jm-commentary_amd/csrc clean
	$(MAKE) -C h264-jm-commentary_amd/host clean
	$(MAKE) -C oracle clean
	$(MAKE) -C tests/harness clean
