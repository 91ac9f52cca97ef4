import json
for f in ['q_bench20', 'q_bench1000', 'q_fov']:
    try:
        d = json.load(open('gpurun_out/' + f + '.json'))
    except Exception as e:
        print(f, 'missing', e)
        continue
    r = d['roofline']
    print(f, round(d['value'] / 1e6, 2), 'us/step', round(d['ms_per_step'] * 1e3, 1), 'kavg', round(r['kernel_avg_us'], 1),
          'bracket', round(r.get('kernel_event_bracket_avg_us', 0), 1), 'kmax', round(r['kernel_max_us'], 1),
          d['status_hist'], d['newton_steps_per_qp'] if f != 'q_bench20' else '')
