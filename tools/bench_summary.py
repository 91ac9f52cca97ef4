import json,sys,os,glob
for p in sorted(glob.glob(sys.argv[1]+'/*.json')):
    l=[x for x in open(p) if x.startswith('{')]
    if not l: print(os.path.basename(p),"no json", open(p[:-5]+".err").read()[-400:]); continue
    d=json.loads(l[-1]); r=d['roofline']; n=d.get('newton_steps_per_qp',{})
    print(os.path.basename(p), '%.3e'%d['value'], 'ms/step %.4f'%d['ms_per_step'], 'p99 %.4f'%d['p99_step_ms'], 'kern %.1f max %.1f'%(r['kernel_avg_us'], r['kernel_max_us']), r['kernel'], {k:v for k,v in d['status_hist'].items() if v}, n.get('max', ''))
    if 'kernel_us_by_step' in n and len(sys.argv)>2: print('   ', n['kernel_us_by_step']); print('   ', n['max_by_step'])
