"""Per-kernel SQ level/instruction ratios (SQ_INST_LEVEL_VMEM / SQ_INSTS_VMEM_RD, LDS, IFETCH) and
SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES from one --pmc pass per workload (round 5: conv_m16q at one
frame vs conv_m16, and the headline).  usage: python tools/sq_levels.py  (reads gpurun_out/lat_r05x/*)"""
import csv,collections,sys
for sub in ('b1','b1m16','head'):
    p='gpurun_out/lat_r05x/%s/run_counter_collection.csv'%sub
    acc=collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(p)):
        k=r['Kernel_Name'].split('(')[0].replace('void ','')[-42:]
        acc[k][r['Counter_Name']]+=float(r['Counter_Value'])
    print('==',sub)
    items=sorted(acc.items(), key=lambda kv:-kv[1].get('SQ_WAVE_CYCLES',0))[:6]
    for k,c in items:
        vm=c['SQ_INST_LEVEL_VMEM']/max(c['SQ_INSTS_VMEM_RD'],1)
        ld=c['SQ_INST_LEVEL_LDS']/max(c['SQ_INSTS_LDS'],1)
        fe=c['SQ_IFETCH_LEVEL']/max(c['SQ_IFETCH'],1)
        print('%-42s vmem_lat %7.1f lds_lat %6.1f ifetch_lat %6.1f ifetch/wavecyc %.4f wait_inst %.3f'%(k,vm,ld,fe,c['SQ_IFETCH']/max(c['SQ_WAVE_CYCLES'],1),c['SQ_WAIT_INST_ANY']/max(c['SQ_WAVE_CYCLES'],1)))
