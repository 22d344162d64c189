# Build / test / bench entry points (reference: Makefile + package.json "test").
PY ?= python

.PHONY: build test test-gpu lint sanitize bench bench-configs verify-bench docker clean

build:            ## host C++ module, gfx950 HIP module, blobd bench peer
	$(PY) -m downloader_amd.ops.build

test: build       ## CPU tier (what CI runs on every push)
	$(PY) -m pytest tests -q -m "not gpu"

test-gpu: build   ## MI355X tier
	$(PY) -m pytest tests -q -m gpu

lint:
	$(PY) -m downloader_amd.utils.lint downloader_amd tests bench.py __graft_entry__.py

sanitize:         ## ASan/UBSan + TSan self-test of the native host code
	$(PY) -m pytest tests/test_native_sanitizers.py -q

bench: build      ## headline: BASELINE config 2 (MB/s staged + p50 latency)
	$(PY) bench.py --steps 16 --warmup 2 --compare-reference

bench-configs: build
	$(PY) -m downloader_amd.bench.configs --config 1 --config 3 --config 4 --config 5

verify-bench: build
	$(PY) -m downloader_amd.bench.verify_bench --gib 4 --piece-mb 1

docker:
	docker build -t downloader-amd .

clean:
	$(PY) -c "from downloader_amd.ops import build; build.clean()"
