"""MFMA-busy evidence per kernel from a rocprofv3 --pmc pass.

The pass (one run, counters within the gfx950 slot limits: 8 SQ, 2 GRBM):
    rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY \
        SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d DIR -- python3 bench.py ...
This script averages every counter per dispatch of each (kernel, grid) and derives
    mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 256 CUs x 4 SIMDs)
the share of the dispatch's active cycles in which an average SIMD's matrix pipe was busy
(GRBM_GUI_ACTIVE is summed over the 8 XCDs: MI355X_MICROARCH.md "DVFS give-back";
SQ_VALU_MFMA_BUSY_CYCLES counts cycles, 16 per v_mfma_f32_16x16x32_f16: § Per-instruction
cycle constants), and the clock the dispatch ran at, GRBM_GUI_ACTIVE / 8 / duration, where
the kernel trace of the same run gives the duration.
usage: python tools/pmc_mfma.py OUT.json CONFIG=DIR [CONFIG=DIR ...]
(the named kernels of each config: NAMED below, kernel-name prefix [| grid])"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SIMDS = 256 * 4


def short(n):
    n = n.replace('void ', '').replace('(anonymous namespace)::', '')
    return n.split('(')[0]


def load(src):
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for f in glob.glob(f'{src}/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            k = f'{short(r["Kernel_Name"])}|{r["Grid_Size"]}'
            acc[k][r['Counter_Name']] += float(r['Counter_Value'])
            disp[k].add((f, r['Dispatch_Id']))
    out = {}
    for k, cs in acc.items():
        n = len(disp[k])
        row = {c: v / n for c, v in cs.items()}
        row['dispatches'] = n
        gui = row.get('GRBM_GUI_ACTIVE')
        if gui and 'SQ_VALU_MFMA_BUSY_CYCLES' in row:
            row['mfma_busy'] = round(row['SQ_VALU_MFMA_BUSY_CYCLES'] / (gui / 8 * SIMDS), 4)
        if 'SQ_WAVE_CYCLES' in row and row['SQ_WAVE_CYCLES'] > 0:
            for c in ('SQ_WAIT_ANY', 'SQ_ACTIVE_INST_ANY'):
                if c in row:
                    row[c.lower() + '_share'] = round(row[c] / row['SQ_WAVE_CYCLES'], 4)
        out[k] = row
    return out


# the kernels the north star names, per bench config (prefix of "name|grid" keys)
NAMED = {
    'c3': {'decoder_lstm': 'rnn_bidir_kernel<1, 512,',
           'postnet_gru': 'rnn_bidir_kernel<0, 256, 8,',
           'prenet_gru': 'rnn_bidir_kernel<0, 256, 16,',
           'prenet_bank': 'conv_gemm_slab_kernel<0, false, true>|1376256',
           'postnet_bank': 'conv_bank_walk_kernel|352256',
           'postnet_proj1': 'conv_gemm_slab_kernel<0, false, true>|528384',
           'postnet_highway_stack': 'highway_stack_kernel<96>',
           'prenet_highway_stack': 'highway_stack_kernel<64>',
           'lstm_input_projection': 'conv_gemm_slabp_kernel<0>|917504'},
    'c2': {'decoder_lstm': 'rnn_gemv_kernel<1, 512,', 'postnet_gru': 'rnn_gemv_kernel<0, 256,',
           'prenet_bank': 'conv_bank_halves_kernel',
           'postnet_highway_stack': 'highway_spread_kernel<3>|106496',
           'prenet_highway_stack': 'highway_spread_kernel<3>|16384'},
    'c5': {'ffn_conv_k9': 'conv_gemm_slab_kernel<0, false, true>|2162688',
           'attention': 'attention_t3_kernel<128, true>',
           'postnet_conv': 'conv_gemm_slab_kernel<0, false, true>|344064'},
}
KEEP = ('mfma_busy', 'SQ_VALU_MFMA_BUSY_CYCLES', 'SQ_BUSY_CYCLES', 'GRBM_GUI_ACTIVE', 'dispatches',
        'sq_wait_any_share', 'sq_active_inst_any_share')


def short_key(k):  # the attention kernel's name stays mangled in the counter CSV
    if k.startswith('_ZN12_GLOBAL__N_119attention_t3_kernelILi128ELb1E'):
        return 'attention_t3_kernel<128, true>' + k[k.index('|'):]
    return k


def main():
    dst = sys.argv[1]
    doc = {'what': __doc__.split('\n\n')[0], 'configs': {}}
    for arg in sys.argv[2:]:
        cfg, src = arg.split('=', 1)
        ks = load(src)
        named = {}
        for name, pref in NAMED.get(cfg, {}).items():
            hit = [(k, v) for k, v in ks.items() if short_key(k).startswith(pref)]
            if hit:
                k, v = max(hit, key=lambda kv: kv[1].get('GRBM_GUI_ACTIVE', 0))
                named[name] = {'kernel': k, **{c: v[c] for c in v if c in KEEP}}
        doc['configs'][cfg] = {'source_dir': src, 'named': named, 'kernels': ks}
        print(f'== {cfg}')
        for name, v in named.items():
            print(f'  {name:24s} busy {v.get("mfma_busy", float("nan")):6.3f}  {v["kernel"][:80]}')
    os.makedirs(os.path.dirname(os.path.abspath(dst)), exist_ok=True)
    json.dump(doc, open(dst, 'w'), indent=1, sort_keys=True)


if __name__ == '__main__':
    main()
