set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03k
O=gpurun_out/r03k
timeout -k 10 300 python -u bench.py --no-cpu --face-model yolov8l-face.pt --frames per-frame --batch 16 --steps 1 --warmup 1 > $O/yolo_pf.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu --face-model yolov8l-face.pt --frames host --batch 16 --steps 1 --warmup 1 > $O/yolo_host.log 2>&1
rc=$?
for f in yolo_pf yolo_host; do echo "== $f"; tail -1 $O/$f.log | cut -c1-900; done
exit $rc
