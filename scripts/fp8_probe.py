import torch, time
print(torch.__version__, hasattr(torch, '_scaled_mm'), torch.cuda.get_device_name(0), torch.cuda.get_device_properties(0).gcnArchName)
for dt in (torch.float8_e4m3fn, torch.float8_e4m3fnuz):
    try:
        a = torch.randn(4096, 896, device='cuda').to(dt)
        b = torch.randn(512, 896, device='cuda').to(dt)
        one = torch.ones((), device='cuda')
        out = torch._scaled_mm(a, b.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
        ref = a.float() @ b.float().t()
        print(dt, 'ok', (out.float() - ref).abs().max().item() / ref.abs().max().item())
        torch.cuda.synchronize(); t=time.time()
        for _ in range(100): torch._scaled_mm(a, b.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
        torch.cuda.synchronize(); print('us', (time.time()-t)*1e4)
        a16, b16 = a.to(torch.bfloat16), b.to(torch.bfloat16)
        torch.cuda.synchronize(); t=time.time()
        for _ in range(100): a16 @ b16.t()
        torch.cuda.synchronize(); print('bf16 us', (time.time()-t)*1e4)
    except Exception as e:
        print(dt, 'fail', repr(e)[:300])
