SHELL=/bin/bash
PY ?= python

.PHONY: native test test-gpu bench bench-configs lint tsan docker clean

native:            ## build the C++ runtime in-tree
	$(PY) -m beholder_amd.ops.build

test: native       ## CPU test suite (what CI runs)
	$(PY) -m pytest tests -q -m "not gpu"

test-gpu: native   ## box-tier tests (full-scale configs)
	$(PY) -m pytest tests -q -m gpu

bench: native      ## headline metric (driver contract)
	$(PY) bench.py

bench-configs: native  ## the five BASELINE.json configs
	$(PY) -m beholder_amd bench all --out profiles/baseline_configs.json

lint:
	@$(PY) -m pyflakes beholder_amd tests bench.py 2>/dev/null || $(PY) -m compileall -q beholder_amd tests bench.py

tsan:              ## ring/framer stress test under ThreadSanitizer + ASan/UBSan
	$(MAKE) -C tests/native run

docker:
	DOCKER_BUILDKIT=1 docker build -t tritonmedia/beholder -f Dockerfile .

clean:
	rm -f beholder_amd/ops/_native*.so beholder_amd/ops/*.srchash
	$(MAKE) -C tests/native clean
