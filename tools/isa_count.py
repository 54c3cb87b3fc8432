"""Count instruction classes per basic block of a kernel in a hipcc -S dump (development)."""
import re, sys, collections
src, pat = sys.argv[1], sys.argv[2]
minlen = int(sys.argv[3]) if len(sys.argv) > 3 else 100
s = open(src).read()
for m in re.finditer(r'^(_Z\w+):', s, re.M):
    if pat not in m.group(1):
        continue
    body = s[m.end():]
    body = body[:body.index('.Lfunc_end')]
    parts = re.split(r'\n(\.LBB\d+_\d+):', body)
    print(m.group(1))
    for i in range(1, len(parts), 2):
        ins = [l.strip().split()[0] for l in parts[i + 1].split('\n')
               if l.strip() and not l.strip().startswith(('.', ';'))]
        if len(ins) < minlen:
            continue
        c = collections.Counter()
        for x in ins:
            k = 'ds' if x.startswith('ds_') else 'v' if x.startswith('v_') else 's' if x.startswith('s_') else 'g' if x.startswith('global') else x
            c[k] += 1
        print(' ', parts[i], len(ins), dict(c))
        print('   ', collections.Counter(x for x in ins if x.startswith(('v_', 's_'))).most_common(30))
