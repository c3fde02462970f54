import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "guetzli-cuda-opencl_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running CPU oracle comparison")


def _ensure_built():
    lib = os.path.join(ROOT, "guetzli-cuda-opencl_amd", "lib", "libguetzli_hip.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-C", os.path.join(ROOT, "guetzli-cuda-opencl_amd", "csrc"),
                        "-j8"], check=True, stdout=subprocess.DEVNULL)
    oracle = os.path.join(ROOT, "oracle", "_build", "libgz_oracle.so")
    if not os.path.exists(oracle):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "oracle"], check=True,
                       stdout=subprocess.DEVNULL)
    occupy = os.path.join(ROOT, "tests", "_build", "libgz_occupy.so")
    src = os.path.join(ROOT, "tests", "native", "occupy.hip")
    if not os.path.exists(occupy) or os.path.getmtime(occupy) < os.path.getmtime(src):
        build_occupy()


def build_occupy():
    """tests/native/occupy.hip -> tests/_build/libgz_occupy.so (a GPU test's
    slot-holding kernel; built here on the CPU, it travels with the tree)."""
    out = os.path.join(ROOT, "tests", "_build", "libgz_occupy.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    tmp = "%s.%d.tmp" % (out, os.getpid())
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-shared", "-fPIC", "--offload-arch=gfx950",
                    os.path.join(ROOT, "tests", "native", "occupy.hip"), "-o", tmp], check=True)
    os.replace(tmp, out)


_ensure_built()


@pytest.fixture(scope="session")
def gz():
    import guetzli_amd
    return guetzli_amd


@pytest.fixture(scope="session")
def gpu_available(gz):
    return gz.device_count() > 0


def _native_bin(name, with_oracle):
    """Builds tests/native/<name>.cc against the product library (and the
    oracle when with_oracle) if missing or stale."""
    out = os.path.join(ROOT, "tests", "_build", name)
    src = os.path.join(ROOT, "tests", "native", name + ".cc")
    lib_dir = os.path.join(ROOT, "guetzli-cuda-opencl_amd", "lib")
    oracle_dir = os.path.join(ROOT, "oracle", "_build")
    host_dir = os.path.join(ROOT, "guetzli-cuda-opencl_amd", "csrc", "host")
    native_dir = os.path.join(ROOT, "tests", "native")
    deps = [src, os.path.join(lib_dir, "libguetzli_hip.so")] + [
        os.path.join(native_dir, f) for f in os.listdir(native_dir) if f.endswith(".h")] + [
        os.path.join(host_dir, f) for f in os.listdir(host_dir) if f.endswith(".h")]
    if not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(d) for d in deps):
        os.makedirs(os.path.dirname(out), exist_ok=True)
        tmp = "%s.%d.tmp" % (out, os.getpid())
        cmd = ["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-pthread",
               "-I", os.path.join(ROOT, "guetzli-cuda-opencl_amd", "csrc"),
               "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "oracle"),
               src, "-o", tmp, "-L", lib_dir, "-lguetzli_hip", "-Wl,-rpath," + lib_dir]
        if with_oracle:
            cmd += ["-L", oracle_dir, "-lgz_oracle", "-Wl,-rpath," + oracle_dir]
        subprocess.run(cmd, check=True)
        # (pytest-xdist workers may build the same binary at once: each links
        # its own file and renames it into place, so none runs a partial one)
        os.replace(tmp, out)
    return out


@pytest.fixture(scope="session")
def strips_e2e_bin():
    """tests/native/strips_oracle_e2e: row strips over threads, oracle comparators."""
    return _native_bin("strips_oracle_e2e", True)


@pytest.fixture(scope="session")
def host_e2e_bin():
    """tests/native/host_oracle_e2e: product host loop + CPU-oracle comparator."""
    return _native_bin("host_oracle_e2e", True)


@pytest.fixture(scope="session")
def lazy_sort_check_bin():
    """tests/native/lazy_sort_check: LazyStdSort vs libstdc++ std::sort."""
    return _native_bin("lazy_sort_check", False)


@pytest.fixture(scope="session")
def collectives_check_bin():
    """tests/native/collectives_check: StagedAllGather (the RCCL collectives'
    buffer handling) over a host-memory transport."""
    return _native_bin("collectives_check", False)


@pytest.fixture(scope="session")
def pool_check_bin():
    """tests/native/pool_check: the shared host worker pool under concurrency."""
    return _native_bin("pool_check", False)


@pytest.fixture(scope="session")
def writer_check_bin():
    """tests/native/writer_check: direct parallel encoder vs SaveToJpegData + WriteJpeg."""
    return _native_bin("writer_check", False)
