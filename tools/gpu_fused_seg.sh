cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for sg in 20 16 24 32; do
  DC_FUSED3=1 DC_FUSED3_SEG=$sg timeout -k 10 300 python3 -u bench.py --no-extra --no-cpu > gpurun_out/fseg_$sg.json 2> gpurun_out/fseg_$sg.err || { tail -20 gpurun_out/fseg_$sg.err; exit 1; }
  python3 -c "
import json;d=[json.loads(l) for l in open('gpurun_out/fseg_$sg.json') if l.startswith('{')][0]
print('seg $sg', d['value'], d['ms_per_step'], d.get('kernels_ms'), d.get('fused_segment_chunks'))"
done
