# tritondl — build / test / bench / package
SHELL      := /bin/bash
PYTHON     ?= python3
ROCM_ARCH  ?= gfx950
IMAGE      ?= tritondl:latest
PYTEST     := $(PYTHON) -m pytest

.PHONY: all build build-force test test-gpu test-all sanitize odr-check bench bench-multi profile-gpu docker-build clean lint

all: build

## build the in-tree native extensions (host C++ hashing + relay, BT peer wire, uTP, HIP gfx950 kernels)
build:
	PYTORCH_ROCM_ARCH=$(ROCM_ARCH) $(PYTHON) tools/build_native.py -v

build-force:
	PYTORCH_ROCM_ARCH=$(ROCM_ARCH) $(PYTHON) tools/build_native.py -v --force

## CPU test suite (what CI and the round driver run)
test: build
	$(PYTEST) tests -x -q -m "not gpu"

## GPU tests (needs an MI355X)
test-gpu: build
	$(PYTEST) tests -x -q -m gpu

test-all: test test-gpu

## native code under ASan+UBSan (host-only; GPU sanitizers are not used)
sanitize:
	$(PYTHON) tools/native_selftest.py --sanitize

## every shared native header linked into two translation units (no non-inline definitions)
odr-check:
	$(PYTHON) tools/odr_check.py

## flagship benchmark (BASELINE config #1), 1 worker
bench: build
	$(PYTHON) bench.py --steps 50 --warmup 5

## 8 workers, one per GPU (torchrun, RCCL for the barriers)
bench-multi: build
	$(PYTHON) -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
	  --master-port 29533 bench.py --gpus 8 --steps 50 --warmup 5

## kernel-level profile of the HIP piece-hash kernels
profile-gpu: build
	cd /tmp && TMPDIR=/tmp rocprofv3 --kernel-trace --stats -d $(CURDIR)/gpurun_out/prof -o hash \
	  --output-format csv -- $(PYTHON) $(CURDIR)/tools/bench_hash.py --no-files

lint:
	$(PYTHON) tools/lint.py

docker-build:
	DOCKER_BUILDKIT=1 docker build -t $(IMAGE) -f docker/Dockerfile .

clean:
	rm -f tritondl/*.so tritondl/*.so.tmp
	find . -name __pycache__ -type d -prune -exec rm -rf {} +
