"""Host sanitizer run of the decoders: `make -C csrc sanitize`
builds decode.cpp + metrics_decode.cpp with -fsanitize=address,undefined
and a mutation fuzzer (csrc/fuzz/decode_fuzz.cpp) that feeds them mutated
golden inputs — including documents above the 64 KiB threshold of the
multi-threaded decode path.  Any out-of-bounds access, use-after-free, leak
or undefined behaviour aborts the run.  No GPU."""
import json
import os
import shutil
import subprocess

import pytest

from conftest import PKG_DIR

CSRC = PKG_DIR / "csrc"


@pytest.fixture(scope="module")
def fuzzer():
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    r = subprocess.run(["make", "-s", "-C", str(CSRC), "sanitize"], capture_output=True, text=True)
    if r.returncode != 0 and "sanitize" in r.stderr and "asan" in r.stderr.lower():
        pytest.skip("no sanitizer runtime: " + r.stderr[-300:])
    assert r.returncode == 0, r.stderr[-2000:]
    return CSRC / "build" / "fuzz" / "decode_fuzz"


def _seeds(golden, tmp_path):
    jd = json.loads((golden / "jaeger_small.json").read_text())
    sw = json.loads((golden / "skywalking_small.json").read_text())["payload"]
    kj = 1 + (80 << 10) // len(json.dumps(jd, indent=2))  # just past the 64 KiB threshold
    ks = 1 + (80 << 10) // len(json.dumps(sw, indent=2))
    big_j = {"data": jd["data"] * kj}
    big_s = dict(sw, traces=sw["traces"] * ks)
    files = {"j_small.json": json.dumps(jd), "j_big.json": json.dumps(big_j, indent=2),
             "s_small.json": json.dumps(sw, indent=2), "s_big.json": json.dumps(big_s, indent=2)}
    for name, text in files.items():
        (tmp_path / name).write_text(text)
    assert (tmp_path / "j_big.json").stat().st_size > 64 << 10
    assert (tmp_path / "s_big.json").stat().st_size > 64 << 10
    return [f"jaeger:{tmp_path / 'j_small.json'}", f"jaeger:{tmp_path / 'j_big.json'}",
            f"skywalking:{tmp_path / 's_small.json'}", f"skywalking:{tmp_path / 's_big.json'}",
            f"long:{golden / 'metric_long.csv'}",
            f"longfile:{golden / 'metric_long.csv'}",
            f"prom:{golden / 'prom_dir' / 'socialnet_container_memory.csv'}",
            f"prom:{golden / 'prom_dir' / 'mongodb_operations_rate.csv'}"]


def test_decoders_under_asan_ubsan(fuzzer, golden, tmp_path, seed=1):
    env = dict(os.environ, ANOMOD_DECODE_THREADS="4", TZ="UTC",
               ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([str(fuzzer), "800", str(seed)] + _seeds(golden, tmp_path), env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    ok, rejected = map(int, r.stdout.split()[1:3])
    assert ok > 100 and rejected > 100  # both outcomes exercised
