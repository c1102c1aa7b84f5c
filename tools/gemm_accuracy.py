"""fp32 GEMM accuracy on this device vs float64 (is torch's device GEMM true fp32?)."""
import torch

torch.manual_seed(0)
a = torch.randn(128, 784, dtype=torch.float64)
w = torch.randn(1000, 784, dtype=torch.float64) * 0.03
ref = a @ w.T
cpu = (a.float() @ w.float().T).double()
print("allow_tf32", torch.backends.cuda.matmul.allow_tf32, "precision", torch.get_float32_matmul_precision())
print("cpu fp32 rel err", ((cpu - ref).abs().max() / ref.abs().max()).item())
for prec in ("highest", "high"):
    torch.set_float32_matmul_precision(prec)
    gpu = (a.float().cuda() @ w.float().cuda().T).double().cpu()
    print(prec, "gpu fp32 rel err", ((gpu - ref).abs().max() / ref.abs().max()).item())
torch.set_float32_matmul_precision("highest")
lin = torch.nn.Linear(784, 1000).cuda()
x = a.float().cuda()
y = lin(x)
yc = torch.nn.functional.linear(x.cpu(), lin.weight.cpu(), lin.bias.cpu())
print("linear fwd gpu vs cpu rel", ((y.cpu() - yc).abs().max() / yc.abs().max()).item())
g = torch.randn_like(y)
y.backward(g)
wg = lin.weight.grad.cpu().double()
wref = g.cpu().double().T @ a
print("weight grad gpu rel err vs fp64", ((wg - wref).abs().max() / wref.abs().max()).item())
