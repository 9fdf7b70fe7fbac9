import torch, time
torch.cuda.init()
x = torch.zeros(1, device="cuda")
for cyc in (10**6, 10**7, 10**8):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); torch.cuda._sleep(cyc); e1.record(); torch.cuda.synchronize()
    print(cyc, e0.elapsed_time(e1), "ms", flush=True)
