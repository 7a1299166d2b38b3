"""Sanitizer runs of the host parsers that take untrusted input: the GGUF reader,
model-config extraction, tokenizer construction and the JSON request parser, built with
AddressSanitizer + UndefinedBehaviorSanitizer (`make sanitize`, csrc/tools/fuzz_host.cpp) and fed
hypothesis-generated corruptions of valid GGUF files and random request bodies.  A clean
rejection (exception) is fine; any sanitizer report fails the test."""
import fcntl
import os
import shutil
import subprocess

import pytest
from hypothesis import HealthCheck, given, settings, strategies as st

from conftest import REPO, make_model

BIN = os.path.join(REPO, "build", "fuzz_host_asan")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")


@pytest.fixture(scope="module")
def fuzz_bin():
    if shutil.which("g++") is None:
        pytest.skip("no host compiler")
    # xdist workers share the binary: serialise the build so none execs a half-linked file
    os.makedirs(os.path.join(REPO, "build"), exist_ok=True)
    with open(os.path.join(REPO, "build", ".sanitize.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        r = subprocess.run(["make", "-s", "sanitize"], cwd=REPO, capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip("sanitizer build failed: " + r.stderr[-300:])
    return BIN


def run(bin_, mode, paths):
    r = subprocess.run([bin_, mode] + list(paths), capture_output=True, text=True, errors="replace", env=ENV,
                       timeout=120)
    report = r.stderr
    assert "AddressSanitizer" not in report and "runtime error" not in report, report[-3000:]
    assert r.returncode == 0, (r.returncode, report[-2000:])
    return r.stdout.splitlines()


@pytest.fixture(scope="module")
def models(native, model_dir):
    return [make_model(model_dir, "tiny-l3", "Q8_0")[0], make_model(model_dir, "tiny-gqa", "Q4_K_M")[0]]


def test_valid_models_parse(fuzz_bin, models):
    out = run(fuzz_bin, "gguf", models)
    assert all(line.startswith("ok") for line in out), out


mutation = st.tuples(st.sampled_from(["flip", "trunc", "stomp", "insert"]), st.floats(0, 1), st.binary(min_size=1, max_size=16))


@settings(max_examples=60, deadline=None, suppress_health_check=list(HealthCheck))
@given(muts=st.lists(mutation, min_size=1, max_size=4), which=st.integers(0, 1), head=st.booleans())
def test_corrupted_gguf(fuzz_bin, models, tmp_path_factory, muts, which, head):
    data = bytearray(open(models[which], "rb").read())
    for kind, where, blob in muts:
        # most structure (header, metadata, tensor table) lives in the first KiBs: bias there
        span = min(len(data), 64 << 10) if head else len(data)
        pos = int(where * max(1, span - 1))
        if kind == "flip":
            data[pos] ^= blob[0] or 0x80
        elif kind == "trunc":
            del data[max(8, pos):]
        elif kind == "stomp":
            data[pos:pos + len(blob)] = blob
        else:
            data[pos:pos] = blob
    p = tmp_path_factory.mktemp("fz") / "m.gguf"
    p.write_bytes(bytes(data))
    run(fuzz_bin, "gguf", [str(p)])


json_text = st.one_of(
    st.text(max_size=200),
    st.recursive(st.none() | st.booleans() | st.floats(allow_nan=False) | st.text(max_size=20),
                 lambda c: st.lists(c, max_size=5) | st.dictionaries(st.text(max_size=8), c, max_size=5),
                 max_leaves=20).map(lambda v: __import__("json").dumps(v)),
)


@settings(max_examples=60, deadline=None, suppress_health_check=list(HealthCheck))
@given(body=json_text, cut=st.integers(0, 400))
def test_json_bodies(fuzz_bin, tmp_path_factory, body, cut):
    p = tmp_path_factory.mktemp("fj") / "b.json"
    p.write_bytes(body.encode("utf-8", "surrogatepass")[: cut or None])
    run(fuzz_bin, "json", [str(p)])
