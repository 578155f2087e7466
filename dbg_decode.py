import sys; sys.path.insert(0, '.')
import numpy as np
from flac_raster_amd import _native
from oracle import oracle as O
ref = open('tests/golden/sample_rgb.flac', 'rb').read()
frames = ref[86:]
with _native.Context(0) as ctx:
    pcm = ctx.decode_frames_host(frames, [0, len(frames)], [65536], channels=3, bps=16)
o = O.decode_frames(frames, 3, 16, 70000)
d = np.argwhere(pcm != o)
print('mismatches', len(d))
for i, c in d[:20]:
    print('sample', i, 'frame', i // 4096, 'off', i % 4096, 'ch', c, 'gpu', pcm[i, c], 'orc', o[i, c])
bad = sorted(set((int(i) // 4096, int(c)) for i, c in d))
print('bad (frame,ch):', bad[:60])
