"""Developer tool: A/B of library builds on one GPU box, interleaved.

Runs bench.py (no CPU leg) once per library per round, alternating, with RTW_LIB
pointing at each build, and prints every ms_per_step and the per-library mean.
usage: python tools/libab.py ROUNDS LIB [LIB ...]   (extra bench.py flags: $LIBAB_ARGS)
A LIB may carry environment settings for its runs: ab/x/librtw.so@RTW_AB=1,RTW_LISTS=1
"""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def libname(spec):
    """ab/<name>/librtw.so[@ENV] -> <name>[@ENV]"""
    lib, _, env = spec.partition("@")
    n = os.path.basename(os.path.dirname(os.path.abspath(lib))) or os.path.basename(lib)
    return n + ("@" + env if env else "")


def lib_env(spec):
    lib, _, env = spec.partition("@")
    extra = dict(kv.split("=", 1) for kv in env.split(",") if kv)
    return dict(os.environ, RTW_LIB=os.path.abspath(lib), **extra)


def main():
    rounds = int(sys.argv[1])
    libs = sys.argv[2:]
    res = {lib: [] for lib in libs}
    for r in range(rounds):
        for lib in libs:
            env = lib_env(lib)
            p = subprocess.run([sys.executable, os.path.join(HERE, "bench.py"), "--steps", "3", "--warmup", "1",
                                "--cpu-baseline", "0", "--pmc", "0", "--e2e", "0"] + os.environ.get("LIBAB_ARGS", "").split(), env=env, capture_output=True, text=True, timeout=300)
            line = [x for x in p.stdout.splitlines() if x.startswith("{")]
            if p.returncode != 0 or not line:
                print(f"{lib}: failed rc={p.returncode}\n{p.stderr[-2000:]}", flush=True)
                sys.exit(1)
            d = json.loads(line[-1])
            ms = d["ms_per_step"]
            res[lib].append(ms)
            par = (d.get("parity") or {}).get("fb_sha256_ok")
            visits = (d.get("stats") or {}).get("node_visits_per_segment")
            print(f"round {r} {libname(lib)}: {ms:.2f} ms  parity {par}  visits/seg {visits}", flush=True)
    for lib, v in res.items():
        print(f"{libname(lib)}: mean {sum(v) / len(v):.2f} ms  {['%.2f' % x for x in v]}")


if __name__ == "__main__":
    main()
