# Build / test / package entry points (reference counterpart: Makefile).
PYTHON    ?= python3
REGISTRY  ?= registry.example.com/amd
VERSION   ?= v0.1.0
GPURUN    ?= /usr/local/graft/bin/gpurun
JOBS      ?= 8

.PHONY: all native test test-gpu bench smoke manifests check-manifests validate-helm-values \
        images image-operator image-node image-driver bundle must-gather e2e clean

all: native test

native:                      ## compile every HIP/C++ component for gfx950 (in-tree)
	$(PYTHON) -m gpu_operator_amd._build -j $(JOBS)

test: native                 ## CPU suite (fake clients, fake sysfs, gloo multi-process)
	$(PYTHON) -m pytest tests/ -x -q -m "not gpu"

test-gpu: native             ## GPU suite on an MI355X box
	$(GPURUN) --timeout 900 -- 'timeout -k 10 600 python -m pytest tests/ -x -q -m gpu'

bench: native
	$(PYTHON) bench.py

smoke: native
	$(PYTHON) __graft_entry__.py smoke

manifests:                   ## regenerate CRD, operator RBAC, OLM CSV
	$(PYTHON) tools/gen_manifests.py

check-manifests:
	$(PYTHON) tools/gen_manifests.py --check

validate-helm-values:        ## render the chart and validate the ClusterPolicy + images
	$(PYTHON) -m gpu_operator_amd.cmd.gpuop_cfg validate clusterpolicy --chart deployments/amd-gpu-operator

images: image-operator image-node image-driver

image-operator:
	docker build -f docker/Dockerfile -t $(REGISTRY)/amd-gpu-operator:$(VERSION) .

image-node:
	docker build -f docker/Dockerfile.node -t $(REGISTRY)/amd-gpu-operator-node:$(VERSION) .

image-driver:
	docker build -f docker/Dockerfile.driver -t $(REGISTRY)/amdgpu-driver:6.12.12 .

bundle: check-manifests
	docker build -f docker/bundle.Dockerfile -t $(REGISTRY)/amd-gpu-operator-bundle:$(VERSION) .

must-gather:
	hack/must-gather.sh

e2e:                         ## against the current kubectl context (one MI355X node)
	tests/e2e/end-to-end.sh

clean:
	rm -rf gpu_operator_amd/_native build *.egg-info
