"""files_len ingestion: the reference's `name<TAB>len` table (V1:301-317)."""
import os

import numpy as np

from partiallyshuffledistributedsampler_amd.files_len import parse_files_len, write_files_len


def test_parse_matches_reference_format(tmp_path):
    base = str(tmp_path)
    with open(os.path.join(base, "files_len_dict"), "w") as f:
        f.write("a.npz\t10\r\nsub/b.npz\t7\n c.npz\t3\n\nafter_blank.npz\t99\n")
    d = parse_files_len(base, "files_len_dict")
    # keys joined onto base_path, values int, reading stops at the first empty line
    assert d == {os.path.join(base, "a.npz"): 10, os.path.join(base, "sub/b.npz"): 7,
                 os.path.join(base, " c.npz"): 3}


def test_roundtrip_feeds_the_sampler(tmp_path):
    from partiallyshuffledistributedsampler_amd.DistributedSamplerViaLocallyShuffleV2 import \
        DistributedSamplerViaLocallyShuffle
    base = str(tmp_path)
    lens = {os.path.join(base, "f%02d.npz" % i): int(n)
            for i, n in enumerate(np.random.default_rng(3).integers(5, 50, 20))}
    write_files_len(base, "files_len_dict", lens)
    fl = parse_files_len(base, "files_len_dict")
    assert fl == lens

    class DS:
        files = list(lens)

        def reset(self):
            pass
    s = DistributedSamplerViaLocallyShuffle(DS(), lambda p, get_data=False: lens[p], num_replicas=2,
                                            rank=0, shuffle_buffer=16, total_size=1, files_len=fl,
                                            device="cpu")
    assert len(s) == -(-sum(lens.values()) // 2)
