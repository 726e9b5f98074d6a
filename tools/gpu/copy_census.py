"""Where the small device copies of one DGETRF come from: torch.Tensor.copy_ / clone / __setitem__ / .to calls during
one getrf_1d factorisation, counted per calling line (python tools/gpu/copy_census.py [N])."""
import collections
import sys
import traceback
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch  # noqa: E402

import dplasma_amd as dp  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
ctx = dp.init(device="cuda:0")
A = dp.block_cyclic(ctx, torch.float64, 512, 512, N, N)
dp.plrnt(ctx, A, 3872)
IP = dp.ipiv_descriptor(ctx, A)
tp = dp.getrf_1d_New(ctx, A, IP)
cnt = collections.Counter()
orig = {}


def wrap(name):
    f = getattr(torch.Tensor, name)
    orig[name] = f

    def g(self, *a, **k):
        if self.is_cuda:
            st = traceback.extract_stack(limit=4)[-2]
            cnt[(name, Path(st.filename).name, st.lineno, st.line)] += 1
        return f(self, *a, **k)
    setattr(torch.Tensor, name, g)


for n in ("copy_", "clone", "__setitem__", "zero_", "fill_", "to", "contiguous"):
    wrap(n)
tp.execute(ctx)
torch.cuda.synchronize()
for n, f in orig.items():
    setattr(torch.Tensor, n, f)
print(f"N={N} steps={A.nt}")
for k, v in cnt.most_common(25):
    print(f"{v:6d}  {k[0]:12s} {k[1]}:{k[2]}  {k[3]}")
