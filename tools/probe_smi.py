import torch, amdsmi, json
h = torch.cuda._get_amdsmi_handler(torch.device("cuda:0"))
for fn in ("amdsmi_get_power_info", "amdsmi_get_gpu_metrics_info", "amdsmi_get_gpu_activity"):
    try:
        r = getattr(amdsmi, fn)(h)
        print(fn, json.dumps({k: (v if isinstance(v, (int, float, str)) or v is None else str(v)[:80]) for k, v in r.items()}))
    except Exception as e:
        print(fn, "ERR", e)
for a in ("power_draw", "clock_rate", "temperature", "utilization"):
    try:
        print(a, getattr(torch.cuda, a)())
    except Exception as e:
        print(a, "ERR", e)
