import sys; sys.path.insert(0, '.')
import bench, octreeraytracer_amd as ort, torch
for cfg in ("ref_stats114", "ref_default"):
    W, H, N, D, M, NS, MD = bench.CONFIGS[cfg]
    r = ort.Renderer(0); r.build_scene(ort.random_spheres(N, 42), D, M)
    p = ort.FrameParams.default_camera(W, H, num_samples=NS, max_depth=MD)
    out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    for _ in range(10): r.render(p, out=out)
    torch.cuda.synchronize()
    print(cfg, [(round(a, 3), b) for a, b in r.frame_trace_times_ms(10)], flush=True)
