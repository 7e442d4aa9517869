# JPEG input step timing (GPU box): 1080p 4:2:0 q90 synthetic JPEGs,
# sift_mi_decode_jpeg per frame (host entropy decode + GPU reconstruction).
import io, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "sift-features_amd"))
import pkg_loader, synth
from PIL import Image
pkg = pkg_loader.load()
ctx = pkg.Context(0)
frames = synth.frames(8, 1920, 1080, seed0=0)
datas = []
for f in frames:
    rgb = np.stack([f, np.roll(f, 5, 1), 255 - f], -1)
    b = io.BytesIO(); Image.fromarray(rgb).save(b, "JPEG", quality=90, subsampling=2); datas.append(b.getvalue())
print("mean JPEG bytes", np.mean([len(d) for d in datas]))
for d in datas[:2]: ctx.decode_jpeg(d)
t = time.perf_counter(); n = 0
for r in range(3):
    for d in datas: ctx.decode_jpeg(d); n += 1
dt = (time.perf_counter() - t) / n
print(f"decode_jpeg 1080p: {dt*1e3:.2f} ms/frame = {1/dt:.0f} frames/s (one host thread)")
t = time.perf_counter()
for d in datas: pkg.jpeg_dims(d)
print(f"headers only: {(time.perf_counter()-t)/len(datas)*1e6:.1f} us/frame")
