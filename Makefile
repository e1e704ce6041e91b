# arena_amd build entry points (reference: Makefile:22-62 builds the static Go binaries).
#   make            build the HIP extension (gfx950) + the native runtime tools
#   make test       CPU test suite (no GPU needed)
#   make test-gpu   GPU tests (MI355X)
#   make bench      flagship benchmark, 1 GPU
#   make test-asan  CPU runtime tests with ASan+UBSan native tools (test-tsan: ThreadSanitizer)
PYTHON ?= python3
export PYTORCH_ROCM_ARCH ?= gfx950

.PHONY: all ext native native-asan native-tsan test test-asan test-tsan test-gpu bench e2e clean version

all: ext native

ext:
	$(PYTHON) setup.py build_ext --inplace

native:
	$(PYTHON) -c 'from arena_amd import _build; print("\n".join(_build.build_native_tools(force=True)))'

# host-code sanitizers for the native runtime tools; GPU code is never sanitized
native-asan:
	$(PYTHON) -c 'from arena_amd import _build; print("\n".join(_build.build_native_tools(force=True, sanitize="asan")))'

native-tsan:
	$(PYTHON) -c 'from arena_amd import _build; print("\n".join(_build.build_native_tools(force=True, sanitize="tsan")))'

test-asan: native-asan
	ARENA_NATIVE_SANITIZE=asan $(PYTHON) -m pytest tests/test_local_backend.py tests/test_parallel.py tests/test_sanitizers.py -q -m "not gpu"

test-tsan: native-tsan
	ARENA_NATIVE_SANITIZE=tsan $(PYTHON) -m pytest tests/test_local_backend.py tests/test_parallel.py tests/test_sanitizers.py -q -m "not gpu"

test:
	$(PYTHON) -m pytest tests -q -m "not gpu"

test-gpu: all
	$(PYTHON) -m pytest tests -q -m gpu

bench: all
	$(PYTHON) bench.py

e2e: all
	bash tools/e2e_mnist.sh

version:
	$(PYTHON) -m arena_amd version

clean:
	rm -rf build arena_amd/_C*.so arena_amd/bin
