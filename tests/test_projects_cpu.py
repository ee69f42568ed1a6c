"""Project entrypoints on CPU: the sort demo learns the task, generate runs end to end."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load(rel):
    spec = importlib.util.spec_from_file_location(os.path.basename(rel)[:-3], os.path.join(ROOT, rel))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_sort_demo_learns():
    tr_acc, te_acc = _load("projects/demo/sort_demo.py").main(["--device", "cpu", "--iters", "300"])
    assert tr_acc > 0.8 and te_acc > 0.8


def test_generate_random_init():
    outs = _load("projects/generate/generate.py").main(
        ["--random-init", "--model-type", "gpt-micro", "--num-samples", "2", "--steps", "4", "--device", "cpu"])
    assert len(outs) == 2
