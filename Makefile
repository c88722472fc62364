# Developer entry points (reference: Makefile / taskfile.yaml targets build, test, manifests,
# bundle, images).  Everything runs from the repository root.
PYTHON ?= python3
REGISTRY ?= dpu-operator-amd
BASE ?= rocm/pytorch:latest
IMAGES := operator daemon vsp-gpu nri p4rt-server cp-agent
GPURUN ?= /usr/local/graft/bin/gpurun

.PHONY: all build test test-gpu bench manifests verify-manifests images bundle clean

all: build

# HIP extension (gfx950), C++ agent module, static dpu-cni + dpu-cp-agent binaries
build:
	$(PYTHON) -m dpu_operator_amd.native.build -v

# CPU suite (control plane, CNI, agent, oracle, gloo multi-process)
test: build
	$(PYTHON) -m pytest tests -q -m "not gpu" -n 4

# GPU suite (MI355X): every kernel is checked bit-exactly against the C++ oracle
test-gpu: build
	$(PYTHON) -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread

bench: build
	$(PYTHON) bench.py --steps 50

# kustomize config/, examples/, OLM bundle/ generated from the code
manifests:
	$(PYTHON) -m dpu_operator_amd.manifests --out . --registry $(REGISTRY)

verify-manifests:
	$(PYTHON) -m pytest tests/test_manifests.py -q

images:
	for t in $(IMAGES); do docker build --build-arg BASE=$(BASE) --target $$t -t $(REGISTRY)/$$t:latest . || exit 1; done

bundle: manifests
	docker build -f bundle.Dockerfile -t $(REGISTRY)/bundle:latest .

clean:
	rm -rf build dpu_operator_amd/native/*.so dpu_operator_amd/native/bin
