import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "tests"))
import numpy as np, torch
import test_gpu_yolo_face as T
from person_capture_amd import face_embedder as fe_mod, imageops
from person_capture_amd._lib import WarpDesc, check
from oracle import pipeline as op, cv_ops
os.environ["PERSON_CAPTURE_AMD_PRECISION"] = "f32"; os.environ["PERSON_CAPTURE_AMD_ARCFACE"] = "iresnet50"
class MP:
    def setenv(self, k, v): os.environ[k] = v
fe, o = T._device(MP(), -2.1)
f = T._frames([0])[0]
im = fe._upload(f, "dbg")
H0, W0 = f.shape[:2]
for ang in (45,):
    M = op.rotation_matrix_2d(W0 / 2.0, H0 / 2.0, ang, 1.0)
    ref = cv_ops.warp_affine(f, M.reshape(-1), W0, H0, border=114 << 8)
    buf = fe._ctx.scratch("yf_affine_dbg", W0 * H0 * 3)
    d = imageops.warp_desc(im.ptr, im.stride, W0, H0, M.reshape(-1), buf.ptr, out_w=W0, out_h=H0, border=imageops.border_constant(114))
    check(fe._ctx.lib.pc_warp_affine(fe._ctx.handle, (WarpDesc * 1)(d), 1), fe._ctx.handle, "w")
    got = fe._ctx.download(buf.ptr, (H0, W0, 3), np.uint8)
    print("affine image diff px", int((got != ref).any(-1).sum()))
    img_r = fe_mod._DevImage(buf.ptr, H0, W0, W0 * 3, buf)
    for ds in (1280, 1536):
        a = fe._yf_predict(img_r, 0.05, ds, 80, iou=0.30)
        b = o.predict(ref, 0.05, ds, 80, iou=0.30)
        print(ds, "dev", len(a[0]), a[0][:2], a[1][:2], "oracle", len(b[0]), b[0][:2], b[1][:2])
r = fe.extract_batch([f])
print("device faces", len(r[0]), [x["bbox"] for x in r[0]])
ro = o.extract(f)
print("oracle faces", len(ro), [x["bbox"] for x in ro], [t for t in o.trace if not t.startswith("predict")])
