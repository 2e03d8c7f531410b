"""files_len ingestion: the reference's `name<TAB>len` file-length table.

The reference's example driver parses it with `parse_files_len(base_path, file_name)`
(DistributedSamplerViaLocallyShuffle.py:301-317): one `name\\tlen` line per file, read until the
first empty line, keys joined onto `base_path`.  The result is the `files_len` dict of the
sampler constructor; files missing from it are probed lazily with reader(path, get_data=False)
in shuffled scan order (V1:186-190, see sampler.py).
"""
import os


def parse_files_len(base_path, file_name, verbose=False):
    """dict {os.path.join(base_path, name): int(len)} of the table `base_path/file_name`.

    Same format and stopping rule as the reference (V1:301-317): lines are `name<TAB>len`,
    stripped of CR/LF, and reading stops at the first empty line."""
    dict_path = os.path.join(base_path, file_name)
    ret = dict()
    with open(dict_path, "r", encoding="utf-8", errors="ignore") as fp:
        if verbose:
            print("parsing file {f}".format(f=dict_path))
        while True:
            line = fp.readline().strip("\n\r")
            if line == "":
                break
            parts = line.split("\t")
            ret[os.path.join(base_path, parts[0])] = int(parts[1])
    if verbose:
        print(str(len(ret)) + " files in " + dict_path)
    return ret


def write_files_len(base_path, file_name, files_len):
    """Write a table parse_files_len reads back (names relative to base_path)."""
    with open(os.path.join(base_path, file_name), "w", encoding="utf-8") as fp:
        for path, n in files_len.items():
            fp.write("%s\t%d\n" % (os.path.relpath(path, base_path), int(n)))
