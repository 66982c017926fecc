import sys, os, json
sys.path.insert(0, "/root/repo/peter-shirley-ray-tracing-the-next-week_amd")
import numpy as np, torch, rtnw
dev = torch.device("cuda", 0)
stream = torch.cuda.current_stream(dev).cuda_stream
out = torch.zeros(500 * 500 * 3, dtype=torch.float32, device=dev)
for scene, cam in (("final", "cornell"), ("cornell_box", "cornell")):
    sc = rtnw.Scene.builtin(scene)
    c = rtnw.Camera.preset(cam, 500, 500)
    for (w, h, spp) in ((1, 1, 1), (8, 8, 1), (64, 64, 1), (500, 500, 1)):
        p = rtnw.RenderParams(500, 500, spp, seed=3)
        ms = []
        for _ in range(5):
            st = sc.render_tiles(c, p, [(0, 0, w, h)], out.data_ptr(), stream)
            ms.append(st["kernel_ms"])
        print(json.dumps({"scene": scene, "tile": [w, h], "spp": spp, "kernel_ms": ms}), flush=True)
    sc.close()
