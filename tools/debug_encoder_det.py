"""Which stage of the fused encoder forward differs between two identical calls (GPU)."""
import torch
import torch.nn.functional as F

from siren_mri_amd import encoder, modules

DEV = torch.device("cuda:0")
torch.manual_seed(4)
enc = modules.ConvImgEncoder(2, (128, 128), hidden_size=128, kernel_size=7, num_conv_res_blocks=2,
                             precision="bf16").to(DEV)
g = torch.Generator().manual_seed(5)
I = torch.randn(2, 2, 128, 128, generator=g).to(DEV)
for mode in ("fused", "chain"):
    encoder.set_fused(mode == "fused")
    outs = []
    for rep in range(3):
        with torch.no_grad():
            outs.append(enc(I).clone())
    print(mode, [torch.equal(outs[0], o) for o in outs[1:]], [(outs[0] - o).abs().max().item() for o in outs[1:]])
encoder.set_fused(True)
# conv alone
x = I.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
w = enc.conv_theta.weight.detach().to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
b = enc.conv_theta.bias.detach().to(torch.bfloat16)
r = [F.conv2d(x, w, b, padding=3) for _ in range(3)]
print("conv_theta", [torch.equal(r[0], t) for t in r[1:]])
t = torch.relu(r[0])
w1 = enc.cnn[0].weight.detach().to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
b1 = enc.cnn[0].bias.detach().to(torch.bfloat16)
r = [F.conv2d(t, w1, b1, padding=3) for _ in range(3)]
print("cnn0", [torch.equal(r[0], t) for t in r[1:]])
a = torch.relu(r[0]).contiguous(memory_format=torch.channels_last)
from siren_mri_amd import _native
lib = _native.lib()
ws = _native.enc_workspace(DEV)
st = _native.stream_handle(DEV)
fw = enc.fc.weight.detach().contiguous()
es = []
for _ in range(5):
    e = torch.empty(2, 128, device=DEV)
    lib.siren_enc_pixfc_fwd(a.data_ptr(), fw.data_ptr(), enc.fc.bias.detach().data_ptr(), e.data_ptr(), 2, 16384, 128,
                            ws.data_ptr(), ws.numel(), st)
    es.append(e)
print("pixfc", [torch.equal(es[0], t) for t in es[1:]])
