"""Debug: large-system training gradients vs the oracle over (H, variants, sizes)."""
import itertools
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_gpu_large_systems as T  # noqa: E402

cases = [([320], 32, 2, {}), ([320], 32, 2, dict(attention=True)), ([320], 32, 2, dict(norm_diff=True, tanh=True)),
         ([320], 64, 2, dict(attention=True, norm_diff=True, tanh=True)), ([100], 32, 2, dict(attention=True)),
         ([320], 128, 1, dict(attention=True))]
for sizes, hid, nl, var in cases:
    try:
        T.test_large_training_gradients_vs_oracle(sizes, hid, nl, var)
        print("OK  ", sizes, hid, nl, var, flush=True)
    except AssertionError as e:
        print("FAIL", sizes, hid, nl, var, str(e)[:300], flush=True)
