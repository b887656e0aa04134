"""Self-synchronisation of the 2-state FSE decoder, in the
pure-Python spec model: decode a C2 block exactly, then start decoders at
random bit offsets with guessed states (0, 0) and count the symbols until
one of them meets the exact decoder (same bit position and both states).
Result on a 64 KiB C2 block: most starts never meet it inside the block
(35 of 40), the rest after 25K-40K symbols -- so speculative segment
decoding cannot replace the sidecar for this format."""
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import spec as S, oracle as O
src = O.generate(0, 0.155, 0x5EED0002, 0, 65536).tobytes()
comp, _ = O.compress2(src)
norm, L, tl, used = S.header_read(comp)
dt = S.decode_table(norm, L, tl)
bits = S.stack_bits(comp[used:])
top = len(bits)
def val(pos, nb):  # bits [pos-nb, pos)
    v = 0
    for i in range(nb):
        v |= bits[pos - nb + i] << i
    return v
pos = top
s0 = val(pos, L); pos -= L
s1 = val(pos, L); pos -= L
# truth trajectory: dict pos -> (a,b) after steps
truth = {}
a, b = s0, s1
p = pos
while True:
    truth[p] = (a, b)
    ns, sym, nb = dt[a]
    if p - nb < 0: break
    v = val(p, nb); p -= nb
    a, b = b, (ns + v) & 0xFFFF
print("truth steps", len(truth), "payload bits", pos)
import random
random.seed(1)
res = []
for trial in range(40):
    start = random.randint(pos // 4, pos * 3 // 4)
    a, b = 0, 0
    p = start
    steps = 0
    while p > 0:
        if p in truth and truth[p] == (a, b):
            break
        ns, sym, nb = dt[a]
        if p - nb < 0: p = -1; break
        v = val(p, nb); p -= nb
        a, b = b, (ns + v) & 0xFFFF
        steps += 1
    res.append(steps if p > 0 else None)
print(sorted(x for x in res if x is not None), res.count(None))
