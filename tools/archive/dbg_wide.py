import sys, random
sys.path.insert(0, '/root/repo')
from biogarden_amd import _device
from biogarden_amd.analysis.seq import edit_distance_batch
for nsym in (129, 200, 230, 250, 255, 256):
    alpha = bytes(range(256 - nsym, 256))
    pairs = [(bytes([x]), bytes([x])) for x in alpha] + [(bytes([x, x]), bytes([x])) for x in alpha]
    d = edit_distance_batch(pairs)
    st = _device.handle().stats()
    bad = [(alpha[i % nsym], i // nsym, d[i]) for i in range(len(pairs)) if d[i] != (i // nsym)]
    print(nsym, st['R'], st['waves'], st['checkpoint'], st['tagged'], len(bad), bad[:4])
