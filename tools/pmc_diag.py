"""Developer tool: extra rocprofv3 --pmc passes over one bench frame (each pass
its own child run, no tracing), per kernel, for the main render kernel's
diagnosis. Reuses bench.py's child and csv reader.

usage: python tools/pmc_diag.py [--size WxH] [--samples-sqrt S] [--mode fast] NAME=CTR,CTR,... [NAME=...]
       (env: RTW_LIB selects a library build, as for bench.py)
prints one JSON object: {pass: {kernel: {counter: value per dispatch}}}
"""
import json
import os
import shutil
import signal
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
import bench  # noqa: E402


def main():
    args = sys.argv[1:]
    size, s = "1200x675", "23"
    if "--size" in args:
        i = args.index("--size")
        size = args[i + 1]
        del args[i:i + 2]
    if "--samples-sqrt" in args:
        i = args.index("--samples-sqrt")
        s = args[i + 1]
        del args[i:i + 2]
    mode = "parity"
    if "--mode" in args:
        i = args.index("--mode")
        mode = args[i + 1]
        del args[i:i + 2]
    exe = shutil.which("rocprofv3")
    out = {}
    tmp = tempfile.mkdtemp(prefix="rtw_pmcdiag_")
    env = dict(os.environ, RTW_NO_TORCH="1")
    try:
        for spec in args:
            name, ctrs = spec.split("=")
            d = os.path.join(tmp, name)
            cmd = [exe, "--pmc", *ctrs.split(","), "-d", d, "-o", "run", "--output-format", "csv", "--",
                   sys.executable, os.path.join(HERE, "bench.py"), "--pmc-child", "--size", size,
                   "--samples-sqrt", s, "--mode", mode]
            p = subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, env=env,
                                 start_new_session=True, cwd=HERE)
            try:
                _, err = p.communicate(timeout=120)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
                p.communicate()
                print(json.dumps({"error": f"pass {name} timed out", **out}))
                sys.exit(1)
            if p.returncode != 0:
                print(json.dumps({"error": f"pass {name} rc {p.returncode}: {err.decode()[-400:]}", **out}))
                sys.exit(1)
            out[name] = bench.read_counters(d)
            print(f"# {name} done", file=sys.stderr, flush=True)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
