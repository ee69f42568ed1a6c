"""The step's epilogue GEMMs at B = 128 (M = 131072 tokens) under every tile config (gemm_set_variant)."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from mingpt_distributed_amd.ops import gemm as G
from mingpt_distributed_amd.ops._ext import ext

C = ext()
M = int(os.environ.get("TOKENS", "131072"))
D = 768
r = lambda *s: (torch.randn(*s, device="cuda") * 0.5).to(torch.bfloat16)


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


x, wfc, bfc = r(M, D), r(4 * D, D), r(4 * D)
u, gd, wp = r(M, 4 * D), torch.empty(M, 4 * D, device="cuda", dtype=torch.bfloat16), r(D, 4 * D)
dz = r(M, D)
wo, y, res = r(D, D), r(M, D), r(M, D)
cases = {
    "fc_fwd_gelu": (lambda: G.gemm_nt(x, wfc, bias=bfc, epi="gelu", pre_out=gd), 2 * M * 4 * D * D),
    "fc_fwd_bias": (lambda: G.gemm_nt(x, wfc, bias=bfc, epi="bias"), 2 * M * 4 * D * D),
    "fc2_dgrad_gelu": (lambda: G.gemm_dgrad(dz, wp, epi="gelu_bwd", aux=gd), 2 * M * 4 * D * D),
    "fc2_dgrad_plain": (lambda: G.gemm_dgrad(dz, wp), 2 * M * 4 * D * D),
    "proj_fwd_resid": (lambda: G.gemm_nt(y, wo, bias=bfc[:D], epi="resid", resid=res, p=0.1, seed=3), 2 * M * D * D),
    "qkv_fwd_bias": (lambda: G.gemm_nt(x, wfc[:3 * D], bias=bfc[:3 * D], epi="bias"), 2 * M * 3 * D * D),
}
if os.environ.get("LMHEAD"):
    wte = r(50304, D)
    cases["lmhead_fwd"] = (lambda: G.gemm_nt(x, wte), 2 * M * 50304 * D)
if os.environ.get("CASES"):
    cases = {k: v for k, v in cases.items() if k in os.environ["CASES"].split(",")}
for v in [int(x) for x in os.environ.get("VARIANTS", "0,1,5,6").split(",")]:
    C.gemm_set_variant(v)
    row = {}
    for k, (fn, fl) in cases.items():
        try:
            t = timeit(fn)
            row[k] = [round(t * 1e3, 1), round(fl / t / 1e9)]
        except Exception as ex:  # noqa: BLE001
            row[k] = str(ex)[:60]
    print(json.dumps({"variant": v, "us_tflops": row}), flush=True)
C.gemm_set_variant(0)
