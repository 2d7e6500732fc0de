"""The legacy-signature compat shim: redrock_old_amd/compat/
rock_serdes_compat.c — desObject / desString / serObject (rock_serdes.h:47-55) plus batch forms —
compiled as C with a minimal Redis model (tests/c/miniredis) into C test programs that run every
golden fixture through the legacy signatures.  CPU: the host-codec route (RedRock's per-key calls,
a fork child's calls) end to end.  GPU: the same fixtures through the GPU route, equal objects and
blobs, and the process exit with foreign threads inside the engine (tests/c/test_compat_exit.c)."""
import json
import os
import struct
import subprocess

import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:   # (run as a script: `python tests/test_compat.py latency`)
    sys.path.insert(0, ROOT)

from helpers import golden  # noqa: E402


def _c_bytes(b):
    return "{" + ",".join(str(x) for x in b) + "}" if b else "{0}"


def write_fixtures(path):
    G = golden()
    fx = G["kats"] + G["edges"]
    lines = ["typedef struct { const char *name; const unsigned char *blob; size_t len; int status;",
             "                 const unsigned char *out; size_t out_len; } fixture_t;"]
    for i, f in enumerate(fx):
        blob = bytes.fromhex(f["blob"])
        out = bytes.fromhex(f.get("reencoded", f["blob"]))
        if len(out) >= 5:   # serObject writes robj.lru: 24 bits (server.h:592-599)
            out = out[:1] + struct.pack("<I", struct.unpack_from("<I", out, 1)[0] & 0xFFFFFF) + out[5:]
        lines.append(f"static const unsigned char B{i}[] = {_c_bytes(blob)};")
        lines.append(f"static const unsigned char O{i}[] = {_c_bytes(out)};")
    lines.append(f"#define N_FIXTURES {len(fx)}")
    lines.append("static const fixture_t FIXTURES[N_FIXTURES] = {")
    for i, f in enumerate(fx):
        blob = bytes.fromhex(f["blob"])
        out_len = len(bytes.fromhex(f.get("reencoded", f["blob"])))
        lines.append(f'  {{"{f["name"]}", B{i}, {len(blob)}, {f["value"].get("status", 0)}, O{i}, {out_len}}},')
    lines.append("};")
    with open(path, "w") as fh:
        fh.write("\n".join(lines) + "\n")


def build(tmp, prog="test_compat"):
    write_fixtures(os.path.join(tmp, "fixtures.h"))
    exe = os.path.join(tmp, prog)
    cmd = ["gcc", "-std=gnu11", "-O1", "-Wall", "-Werror", "-Wno-unused-function", "-DRR_REDIS_TREE",
           "-I", os.path.join(ROOT, "tests", "c", "miniredis"), "-I", os.path.join(ROOT, "include"), "-I", tmp,
           os.path.join(ROOT, "redrock_old_amd", "compat", "rock_serdes_compat.c"),
           os.path.join(ROOT, "tests", "c", "miniredis", "miniredis.c"),
           os.path.join(ROOT, "tests", "c", prog + ".c"),
           "-L", os.path.join(ROOT, "redrock_old_amd"), "-lrr_serdes", "-lpthread",
           "-Wl,-rpath," + os.path.join(ROOT, "redrock_old_amd"), "-o", exe]
    subprocess.run(cmd, check=True)
    return exe


def test_compat_shim_builds_as_c(tmp_path):
    exe = build(str(tmp_path))
    assert os.path.exists(exe)
    nm = subprocess.run(["nm", exe], capture_output=True, text=True, check=True).stdout
    for sym in ("desObject", "desString", "serObject", "rr_compat_des_batch", "rr_compat_ser_batch"):
        assert f" T {sym}" in nm, sym


def build_link(tmp):
    """tests/c/test_rock_link.c: rock_serdes.h:47-55 exactly as rock.c sees them, linked against
    the shim + the Redis model + librr_serdes.so."""
    exe = os.path.join(tmp, "test_rock_link")
    cmd = ["gcc", "-std=gnu11", "-O1", "-Wall", "-Werror", "-Wno-unused-function", "-DRR_REDIS_TREE",
           "-I", os.path.join(ROOT, "tests", "c", "miniredis"), "-I", os.path.join(ROOT, "include"),
           os.path.join(ROOT, "redrock_old_amd", "compat", "rock_serdes_compat.c"),
           os.path.join(ROOT, "tests", "c", "miniredis", "miniredis.c"),
           os.path.join(ROOT, "tests", "c", "test_rock_link.c"),
           "-L", os.path.join(ROOT, "redrock_old_amd"), "-lrr_serdes", "-lpthread",
           "-Wl,-rpath," + os.path.join(ROOT, "redrock_old_amd"), "-o", exe]
    subprocess.run(cmd, check=True)
    return exe


def test_rock_c_call_set_links(tmp_path):
    """Every function rock_serdes.h:47-55 declares is defined by the shim, so rock.c's call set
    (desObject :468/:538, serObject :691, the ROCK testserdes* hooks :175-183) links unchanged."""
    exe = build_link(str(tmp_path))
    nm = subprocess.run(["nm", exe], capture_output=True, text=True, check=True).stdout
    for sym in ("desString", "serObject", "desObject", "_test_ser_des_string", "_test_ser_des_list",
                "_test_ser_des_set", "_test_ser_des_hash", "_test_ser_des_zset"):
        assert f" T {sym}" in nm, sym


@pytest.mark.gpu
def test_rock_c_call_set_runs_on_gpu(tmp_path):
    exe = build_link(str(tmp_path))
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    print(r.stdout[-4000:], r.stderr[-2000:])
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr
    assert "0 failures" in r.stdout


def test_compat_shim_host_route_cpu(tmp_path):
    """RedRock's per-key calls through the shim with no GPU: every golden fixture through
    desObject / desString / serObject on the host codec (the verdicts, the objects, the bytes
    serObject writes), the batch forms, the fork-child route in-process and through real forks
    (a child forced onto the GPU route refuses instead of touching HIP)."""
    exe = build(str(tmp_path))
    r = subprocess.run([exe, "host"], capture_output=True, text=True, timeout=120)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout


@pytest.mark.gpu
def test_compat_shim_round_trips_fixtures_on_gpu(tmp_path):
    """The host-route checks, then every fixture through the GPU route: the same verdicts, objects
    equal to the host route's, the same blobs; a fork after the parent used the GPU."""
    exe = build(str(tmp_path))
    r = subprocess.run([exe, "gpu"], capture_output=True, text=True, timeout=120)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout and "objects equal: yes" in r.stdout


def test_compat_exit_program_builds(tmp_path):
    assert os.path.exists(build(str(tmp_path), "test_compat_exit"))


@pytest.mark.gpu
def test_compat_exit_with_foreign_threads_in_engine(tmp_path):
    """exit() while one thread's context teardown is held inside the engine
    (test hook, 400 ms) and another thread loops desObject on the GPU route, as RedRock's
    never-joined rock thread does (rock.c:615, :552-596).  The shim's exit handler waits for the
    calls in flight and parks later callers before the HIP runtime's teardown: exit status 0."""
    exe = build(str(tmp_path), "test_compat_exit")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, (r.returncode, r.stdout + r.stderr)
    assert "thread A's teardown held" in r.stdout


# ---- row f4: batched snapshot restore over the fork-child pipes (include/rr_rdb.h) --------
def build_rdb(tmp, bench=False):
    """bench=True links the oracle (test infrastructure) for the CPU desObject legs of the bench."""
    write_fixtures(os.path.join(tmp, "fixtures.h"))
    exe = os.path.join(tmp, "test_rdb")
    oracle = os.path.join(ROOT, "oracle")
    extra = (["-DRR_RDB_BENCH_ORACLE", "-I", oracle, "-L", oracle, "-lrr_oracle", "-Wl,-rpath," + oracle]
             if bench else [])
    cmd = ["gcc", "-std=gnu11", "-O2", "-Wall", "-Werror", "-Wno-unused-function", "-DRR_REDIS_TREE", "-pthread",
           "-I", os.path.join(ROOT, "tests", "c", "miniredis"), "-I", os.path.join(ROOT, "include"), "-I", tmp,
           os.path.join(ROOT, "redrock_old_amd", "compat", "rock_serdes_compat.c"),
           os.path.join(ROOT, "tests", "c", "miniredis", "miniredis.c"),
           os.path.join(ROOT, "tests", "c", "test_rdb.c"),
           "-L", os.path.join(ROOT, "redrock_old_amd"), "-lrr_serdes",
           "-Wl,-rpath," + os.path.join(ROOT, "redrock_old_amd")] + extra + ["-o", exe]
    subprocess.run(cmd, check=True)
    return exe


def test_rdb_batch_protocol_cpu(tmp_path):
    """RAW mode needs no GPU: pipelined batch requests (20000 keys, no deadlock), wire
    compatibility with the reference's serial child and serial service, missing-key exit."""
    exe = build_rdb(str(tmp_path))
    r = subprocess.run([exe, "cpu"], capture_output=True, text=True, timeout=120)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout


@pytest.mark.gpu
def test_rdb_flat_restore_on_gpu(tmp_path):
    """FLAT mode: the service decodes on the GPU, the child builds robj from the records;
    every restored value equals desObject of its blob."""
    exe = build_rdb(str(tmp_path))
    r = subprocess.run([exe, "gpu"], capture_output=True, text=True, timeout=120)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout


def build_callpattern(tmp):
    """tests/c/bench_callpattern.c: the shim inside the reference callers' patterns (evictor: k
    serObject per cycle; restore: k desObject jobs), per-value shim vs batch forms vs the faithful
    CPU restatement (the oracle, linked only into this bench)."""
    exe = os.path.join(tmp, "bench_callpattern")
    oracle = os.path.join(ROOT, "oracle")
    cmd = ["gcc", "-std=gnu11", "-O2", "-Wall", "-Werror", "-Wno-unused-function", "-DRR_REDIS_TREE", "-pthread",
           "-I", os.path.join(ROOT, "tests", "c", "miniredis"), "-I", os.path.join(ROOT, "include"), "-I", oracle,
           os.path.join(ROOT, "redrock_old_amd", "compat", "rock_serdes_compat.c"),
           os.path.join(ROOT, "tests", "c", "miniredis", "miniredis.c"),
           os.path.join(ROOT, "tests", "c", "bench_callpattern.c"),
           "-L", os.path.join(ROOT, "redrock_old_amd"), "-lrr_serdes", "-Wl,-rpath," + os.path.join(ROOT, "redrock_old_amd"),
           "-L", oracle, "-lrr_oracle", "-Wl,-rpath," + oracle, "-lm", "-o", exe]
    subprocess.run(cmd, check=True)
    return exe


def test_callpattern_bench_builds(tmp_path):
    assert os.path.exists(build_callpattern(str(tmp_path)))


def build_latency(tmp):
    """tests/c/bench_latency.c: per-call latency of desObject / serObject through the shim, the
    batch C-ABI with one value per call (one-launch kernels / pipeline), and the faithful CPU
    restatement (the oracle: test infrastructure, linked only into this bench)."""
    exe = os.path.join(tmp, "bench_latency")
    oracle = os.path.join(ROOT, "oracle")
    cmd = ["gcc", "-std=gnu11", "-O2", "-Wall", "-Werror", "-Wno-unused-function", "-DRR_REDIS_TREE", "-pthread",
           "-I", os.path.join(ROOT, "tests", "c", "miniredis"), "-I", os.path.join(ROOT, "include"), "-I", oracle,
           os.path.join(ROOT, "redrock_old_amd", "compat", "rock_serdes_compat.c"),
           os.path.join(ROOT, "tests", "c", "miniredis", "miniredis.c"),
           os.path.join(ROOT, "tests", "c", "bench_latency.c"),
           "-L", os.path.join(ROOT, "redrock_old_amd"), "-lrr_serdes", "-Wl,-rpath," + os.path.join(ROOT, "redrock_old_amd"),
           "-L", oracle, "-lrr_oracle", "-Wl,-rpath," + oracle, "-lm", "-o", exe]
    subprocess.run(cmd, check=True)
    return exe


def test_latency_bench_builds(tmp_path):
    assert os.path.exists(build_latency(str(tmp_path)))


@pytest.mark.gpu
def test_per_value_latency_path(tmp_path):
    """The unchanged per-value callers' path: every desObject / serObject of 300 config-4 values
    on the default route (the host codec) and forced onto the GPU route (the one-launch kernels)
    round-trips (the bench checks every blob)."""
    r = subprocess.run([build_latency(str(tmp_path)), "4", "300"], capture_output=True, text=True, timeout=120)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["roundtrip_bad"] == 0 and line["gpu"]
    assert line["shim_gpu_route_desObject_us"]["median"] > 0 and line["shim_desObject_us"]["median"] > 0


if __name__ == "__main__":   # python tests/test_compat.py bench [config k] | latency [config k] | callpattern [config]  (GPU box)
    import sys
    import tempfile
    if sys.argv[1:2] == ["bench"]:   # keys/s of the restore paths
        with tempfile.TemporaryDirectory() as d:
            r = subprocess.run([build_rdb(d, bench=True), "bench"] + sys.argv[2:4], capture_output=True, text=True,
                               timeout=600)
            print(r.stdout, r.stderr)
    if sys.argv[1:2] == ["callpattern"]:   # the shim in the evictor / restore call patterns
        with tempfile.TemporaryDirectory() as d:
            r = subprocess.run([build_callpattern(d)] + sys.argv[2:3], capture_output=True, text=True, timeout=900)
            print(r.stdout, r.stderr)
    if sys.argv[1:2] == ["latency"]:   # per-call latency of the one-value signatures
        with tempfile.TemporaryDirectory() as d:
            r = subprocess.run([build_latency(d)] + sys.argv[2:4], capture_output=True, text=True, timeout=600)
            print(r.stdout, r.stderr)


# ---- row f2: batched store I/O around the GPU path (include/rr_kv.h) ----------------------
def build_kv(tmp):
    write_fixtures(os.path.join(tmp, "fixtures.h"))
    exe = os.path.join(tmp, "test_kv")
    cmd = ["gcc", "-std=gnu11", "-O1", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), "-I", tmp,
           os.path.join(ROOT, "tests", "c", "test_kv.c"), "-L", os.path.join(ROOT, "redrock_old_amd"), "-lrr_serdes",
           "-Wl,-rpath," + os.path.join(ROOT, "redrock_old_amd"), "-o", exe]
    subprocess.run(cmd, check=True)
    return exe


def test_kv_batch_io_builds(tmp_path):
    exe = build_kv(str(tmp_path))
    nm = subprocess.run(["nm", exe], capture_output=True, text=True, check=True).stdout
    assert " U rr_kv_dump_batch" in nm and " U rr_kv_restore_batch" in nm


@pytest.mark.gpu
def test_kv_batch_io_on_gpu(tmp_path):
    """One WriteBatch-shaped dump and one MultiGet-shaped restore of 3000 values, plain and
    snappy-compressed: stored bytes are serObject's, the restore equals the decode of them."""
    exe = build_kv(str(tmp_path))
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout
