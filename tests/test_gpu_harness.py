"""The reference's own drivers, compiled unchanged against the drop-in headers
(harness/build.sh), run against liblabsort.so.

  main.cpp            warm-up + measured sweep 256..65536 through order_array and
                      order_with_trust, CSV in ./output.txt (main.cpp:17-51)
  performanceTest.cpp order_with_trust sweep, one stdout line per size (:20-49)

LABSORT_VERIFY=1 makes every drop-in call check its own result (no descents, same
multiset as the input) and print "labsort-verify,<caller>,<n>,ok" on stderr -- the
verify column, added without editing main.cpp.  performaceTest only calls the
host-side thrust sort, so it also runs here on CPU."""
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "harness", "bin")
SIZES = [256 << i for i in range(9)]  # main.cpp:24,35 / performanceTest.cpp:25,47: 256 .. 65536


def _exe(name):
    exe = os.path.join(BIN, name)
    if not os.path.exists(exe):
        pytest.skip("harness binaries not built (reference sources absent when building)")
    return exe


def _verify_lines(stderr, who):
    return [int(m.group(1)) for m in re.finditer(rf"^labsort-verify,{who},(\d+),ok$", stderr, re.M)]


def test_performance_test_format_and_verify(tmp_path):
    env = dict(os.environ, LABSORT_VERIFY="1")
    r = subprocess.run([_exe("performaceTest")], cwd=tmp_path, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [x for x in r.stdout.splitlines() if x.strip()]
    # performanceTest.cpp:43  printf("\nSize = %d | Nuestro = ?? | Trust = %.3f ms", ...)
    pat = re.compile(r"^Size = (\d+) \| Nuestro = \?\? \| Trust = (\d+\.\d{3}) ms$")
    got = [pat.match(x) for x in lines]
    assert all(got), lines
    assert [int(m.group(1)) for m in got] == SIZES
    assert _verify_lines(r.stderr, "order_with_trust") == SIZES


def test_performance_test_verify_off(tmp_path):
    env = {k: v for k, v in os.environ.items() if k != "LABSORT_VERIFY"}
    r = subprocess.run([_exe("performaceTest")], cwd=tmp_path, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "labsort-verify" not in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("algo", [None, "radix", "merge"])
def test_main_output_csv_and_verify(tmp_path, algo):
    """main.cpp end to end on the GPU: output.txt has the reference's header and one
    Our + one Trust row per size (main.cpp:21,42-43); every order_array result was
    verified by the library (warm-up and measured calls: 2 x 9)."""
    env = dict(os.environ, LABSORT_VERIFY="1")
    if algo:
        env["LABSORT_ALGO"] = algo
    r = subprocess.run([_exe("sort")], cwd=tmp_path, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    rows = (tmp_path / "output.txt").read_text().splitlines()
    assert rows[0] == "Size,Time,Algorithm"
    body = rows[1:]
    assert len(body) == 2 * len(SIZES)
    for i, size in enumerate(SIZES):
        for j, name in enumerate(("Our", "Trust")):
            s, t, a = body[2 * i + j].split(",")
            assert int(s) == size and a == name
            assert re.fullmatch(r"\d+\.\d{6}", t) and float(t) >= 0.0  # "%f"
    assert _verify_lines(r.stderr, "order_array") == SIZES + SIZES
    assert _verify_lines(r.stderr, "order_with_trust") == SIZES + SIZES
    assert "GPUassert" not in r.stderr
