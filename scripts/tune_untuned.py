"""TunableOp in bounded chunks (one whole-step tuning run of config 5 was killed at 900 s).

Step 1 -- record which library GEMMs of a bench step have no entry in the committed table (no tuning, one
short run; TunableOp writes their signatures to an "untuned" file):

    python scripts/tune_untuned.py record <untuned.csv> -- python bench_configs.py --configs 5 --steps 1 --warmup 1

Step 2 -- tune a slice of those signatures in a process of its own (each slice under its own time limit, so a
slow shape loses only its slice), merging the winners into <out.csv> (created from the committed table):

    python scripts/tune_untuned.py tune <untuned.csv> <out.csv> <start> <count>

Step 3 -- copy <out.csv> over tuning/tunableop_gfx950.csv (utils/tuning.py loads it read-only at run time).
"""
import os
import shutil
import subprocess
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TABLE = os.path.join(ROOT, "tuning", "tunableop_gfx950.csv")


def _entries(path):
    if not os.path.exists(path):
        return []
    return [ln for ln in open(path).read().splitlines() if ln and not ln.startswith("Validator")]


def record(untuned, cmd):
    d = tempfile.mkdtemp(prefix="vcx_rec_")
    shutil.copyfile(TABLE, os.path.join(d, "results0.csv"))
    env = dict(os.environ, PYTORCH_TUNABLEOP_ENABLED="1", PYTORCH_TUNABLEOP_TUNING="0",
               PYTORCH_TUNABLEOP_RECORD_UNTUNED="1", PYTORCH_TUNABLEOP_FILENAME=os.path.join(d, "results%d.csv"),
               PYTORCH_TUNABLEOP_UNTUNED_FILENAME=os.path.join(d, "untuned%d.csv"))
    rc = subprocess.call(cmd, env=env)
    got = _entries(os.path.join(d, "untuned0.csv"))
    seen, out = set(), []
    for ln in got:
        key = tuple(ln.split(",")[:2])
        if key not in seen:
            seen.add(key)
            out.append(ln)
    with open(untuned, "w") as f:
        f.write("\n".join(out) + ("\n" if out else ""))
    print(f"[record] rc={rc}: {len(out)} untuned GEMM signatures -> {untuned}", flush=True)
    return rc


def tune(untuned, out_csv, start, count):
    base = out_csv if os.path.exists(out_csv) else TABLE
    have = {tuple(ln.split(",")[:2]) for ln in _entries(base)}
    todo = [ln for ln in _entries(untuned)[start:start + count] if tuple(ln.split(",")[:2]) not in have]
    print(f"[tune] {len(todo)} signatures (slice {start}..{start + count})", flush=True)
    if not todo:
        return 0
    d = tempfile.mkdtemp(prefix="vcx_tune_")
    shutil.copyfile(base, os.path.join(d, "results0.csv"))
    part = os.path.join(d, "todo.csv")
    with open(part, "w") as f:
        f.write("\n".join(todo) + "\n")
    os.environ["PYTORCH_TUNABLEOP_ENABLED"] = "1"
    os.environ["PYTORCH_TUNABLEOP_TUNING"] = "1"
    os.environ["PYTORCH_TUNABLEOP_FILENAME"] = os.path.join(d, "results%d.csv")
    os.environ.setdefault("PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS", "30")
    os.environ.setdefault("PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS", "10")
    t0 = time.time()

    def beat():  # a big shape tunes for tens of seconds without output of its own
        while True:
            time.sleep(30)
            print(f"[tune] {time.time() - t0:.0f} s", flush=True)

    threading.Thread(target=beat, daemon=True).start()
    import torch

    torch.cuda.set_device(0)
    torch.cuda.tunable.tune_gemm_in_file(part)
    res = torch.cuda.tunable.get_results()
    lines = _entries(base)
    new = [f"{r[0]},{r[1]},{r[2]},{r[3]}" for r in res if (r[0], r[1]) not in have]
    validators = [ln for ln in open(base).read().splitlines() if ln.startswith("Validator")]
    with open(out_csv, "w") as f:
        f.write("\n".join(validators + lines + new) + "\n")
    print(f"[tune] {len(new)} new entries in {time.time() - t0:.0f} s -> {out_csv}", *new, sep="\n", flush=True)
    return 0


if __name__ == "__main__":
    if sys.argv[1] == "record":
        i = sys.argv.index("--")
        sys.exit(record(sys.argv[2], sys.argv[i + 1:]))
    sys.exit(tune(sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5])))
