"""bench_configs.py runs several configs as one child process each (config 4 after config 3 in one process measured
15 % slow, profiles/r6_final_validation.txt): the child's argv keeps every other argument."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load():
    spec = importlib.util.spec_from_file_location("bench_configs", os.path.join(ROOT, "bench_configs.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_child_argv_replaces_configs():
    m = _load()
    assert m.child_argv(["--configs", "3,4", "--steps", "8"], "4") == ["--configs", "4", "--steps", "8"]
    assert m.child_argv(["--steps", "8", "--configs=3,4", "--no-graph"], "3") == ["--configs", "3", "--steps", "8",
                                                                                  "--no-graph"]
    assert m.child_argv([], "5") == ["--configs", "5"]
