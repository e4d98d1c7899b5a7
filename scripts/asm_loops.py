"""Lists the loops of one kernel in a .s file that contain DPP ops, with VALU/SALU/DPP counts."""
import re
import sys

path, pat = sys.argv[1], sys.argv[2]
lines = open(path).read().split('\n')
start = [i for i, l in enumerate(lines) if re.match(r'^_Z\S*' + pat + r'\S*:', l)][0]
end = [i for i in range(start, len(lines)) if 's_endpgm' in lines[i]][0]
body = lines[start:end]
labels = {}
for i, l in enumerate(body):
    m = re.match(r'^(\.LBB\d+_\d+):', l)
    if m:
        labels[m.group(1)] = i
for i, l in enumerate(body):
    m = re.search(r's_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)', l)
    if m and m.group(1) in labels and labels[m.group(1)] < i:
        seg = body[labels[m.group(1)]:i + 1]
        nd = sum(('row_' in x or 'wave_sh' in x or 'quad_perm' in x) for x in seg)
        nv = sum(bool(re.match(r'\s+v_', x)) for x in seg)
        ns = sum(bool(re.match(r'\s+s_', x)) for x in seg)
        nl = sum(bool(re.match(r'\s+ds_', x)) for x in seg)
        if nd or len(sys.argv) > 3:
            print(f"lines {start + labels[m.group(1)] + 1}-{start + i + 1}: valu {nv} salu {ns} dpp {nd} ds {nl}")
