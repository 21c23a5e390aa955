import numpy as np

from metagenomics_amd import synth


def test_generator_deterministic():
    a = synth.uniform_read_set(1000, 100, 5000, seed=11)
    b = synth.uniform_read_set(1000, 100, 5000, seed=11)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_reads_come_from_genome_either_strand():
    g = synth.random_genome(3000, 5)
    gs = synth.codes_to_strings(g[None, :], np.array([3000]))[0]
    c, L = synth.sample_reads(g, 200, 50, 90, seed=6)
    for s in synth.codes_to_strings(c, L):
        assert s in gs or synth.revcomp_str(s) in gs


def test_metagenome_shapes():
    c, L = synth.metagenome_read_set(2000, 100, 250, n_genomes=5, total_len=50000, seed=2)
    assert c.shape[0] == 2000 and L.min() >= 100 and L.max() <= 250
