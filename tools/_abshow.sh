cat gpurun_out/ab.log; tail -2 gpurun_out/q_pytest.log
python3 -c "
import json
for f in ['ab_coll','ab_coll20','ab_8192','ab_fov','ab_fovs']:
    try: d=json.load(open('gpurun_out/'+f+'.json'))
    except Exception as e: print(f, e); continue
    r=d['roofline']; print(f, '%.4g'%d['value'], round(r['kernel_avg_us'],2), round(r['kernel_max_us'],1), d['status_hist'])"
grep -E "^   (setup|neighbours|cbf_rows|solve|outputs)|span" gpurun_out/ab_stamps.log
