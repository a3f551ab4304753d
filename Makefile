# Top-level build: the product (libjmhip.so + host plumbing + lencod) and the test-only oracle.
.PHONY: all product oracle clean
all: product oracle

product:
	$(MAKE) -C h264-jm-commentary_amd/csrc libjmhip.so
	$(MAKE) -C h264-jm-commentary_amd/host all

oracle: product
	$(MAKE) -C oracle all

clean:
	$(MAKE) -C h264-jm-commentary_amd/csrc clean
	$(MAKE) -C h264-jm-commentary_amd/host clean
	$(MAKE) -C oracle clean
