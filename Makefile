SHELL=/bin/bash
PY ?= python

.PHONY: native test test-gpu bench bench-configs lint tsan asan coverage docker clean

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
	$(PY) -m compileall -q beholder_amd tests bench.py
	$(PY) scripts/lint.py beholder_amd tests bench.py __graft_entry__.py scripts

tsan:              ## ring/framer stress test under ThreadSanitizer + ASan/UBSan
	$(MAKE) -C tests/native run

asan:             ## CPython suites against an ASan+UBSan build of the extension (host code only)
	$(PY) -m beholder_amd.ops.build --force --sanitize=address,undefined
	BEHOLDER_ALLOW_BUILD=0 ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=halt_on_error=1 \
	  LD_PRELOAD="$$(gcc -print-file-name=libasan.so) $$(gcc -print-file-name=libubsan.so) $${LD_PRELOAD:-}" \
	  $(PY) -m pytest -q -p no:cacheprovider -m "not gpu" tests/test_native_fuzz.py tests/test_codec.py tests/test_ingest.py \
	  tests/test_amqp_demux.py tests/test_text.py tests/test_delivery.py tests/test_histogram.py \
	  tests/test_handlers.py tests/test_native_handlers.py tests/test_tracing.py tests/test_amqp.py tests/test_service.py tests/test_h1.py tests/test_h1_fast.py tests/test_tls.py tests/test_netconn.py tests/test_sinks.py tests/test_stores.py tests/test_preconnect.py tests/test_driver.py tests/test_chaos.py tests/test_workers.py tests/test_gpu_decode.py tests/test_native_tools.py tests/test_pg_fake.py tests/test_gil_clock.py \
	  tests/test_native_handlers_edges.py tests/test_h1_call_edges.py tests/test_netconn_edges.py tests/test_native_surface.py tests/test_direct_dispatch.py tests/test_reference_oracle.py; \
	  rc=$$?; $(PY) -m beholder_amd.ops.build --force >/dev/null; exit $$rc

coverage:         ## gcov line / branch coverage of the native runtime under the CPU suite -> profiles/native_coverage
	$(PY) scripts/native_coverage.py --out profiles/native_coverage

docker:
	DOCKER_BUILDKIT=1 docker build -t tritonmedia/beholder -f Dockerfile .

clean:
	rm -f beholder_amd/ops/_native*.so beholder_amd/ops/*.srchash
	$(MAKE) -C tests/native clean
