"""bench.py's roofline evidence lookup (CPU): each config's dominant recurrence maps to the
kernel that actually runs (B <= 4: the exact-fp32 GEMV recurrence, rnn.hip gemv_path), and
the committed PMC summaries hold exactly one such kernel."""
import bench


def test_rocprof_name_follows_the_gemv_rule(monkeypatch):
    monkeypatch.delenv('FTMI_RNN_GEMV', raising=False)
    assert bench.rocprof_name('rnn_bidir[lstm,B=1,T=816,H=512,mma=2]') == 'rnn_gemv_kernel<1, 512,'
    assert bench.rocprof_name('rnn_bidir[gru,B=4,T=816,H=256,mma=2]') == 'rnn_gemv_kernel<0, 256,'
    assert bench.rocprof_name('rnn_bidir[lstm,B=64,T=1368,H=512,mma=2]') == 'rnn_bidir_kernel<1, 512,'
    assert bench.rocprof_name('rnn_bidir[gru,B=1,T=816,H=32,mma=2]') == 'rnn_bidir_kernel<0, 32,'
    monkeypatch.setenv('FTMI_RNN_GEMV', '0')
    assert bench.rocprof_name('rnn_bidir[lstm,B=1,T=816,H=512,mma=2]') == 'rnn_bidir_kernel<1, 512,'
    assert bench.rocprof_name('rnn_bidir[gru,B=64,T=200,H=64,mma=2]') == 'rnn_bidir_kernel<0, 64,'
    assert bench.rocprof_name('conv1d[M=12800,N=256,K=1280,mma=2]') is None


def test_committed_traffic_covers_the_dominant_kernels(monkeypatch):
    monkeypatch.delenv('FTMI_RNN_GEMV', raising=False)
    c3 = bench.pmc_traffic('rnn_bidir[lstm,B=64,T=1368,H=512,mma=2]', bench.PMC_PROFILE)
    c2 = bench.pmc_traffic('rnn_bidir[lstm,B=1,T=816,H=512,mma=2]', bench.PMC_PROFILE_C2)
    for t in (c3, c2):
        assert t is not None and t['bytes_per_launch'] > 0
    # c2: W_hh (8.4 MB) + phoneme-rate projections + y: no re-read of the weights per step
    assert c2['bytes_per_launch'] < 2 * 8.4e6


def test_committed_traffic_covers_the_c5_dominant_conv():
    """c5's dominant kernel is a slab-kernel conv: its dispatch is found by grid (whole XCD
    rounds of 256-row tiles x 128-column tiles, 768 threads), and the PMC write bytes equal
    its output exactly (B * T_mel rows x 1024 fp32)."""
    t = bench.pmc_traffic_slab('conv1d[M=89600,N=1024,K=2304,mma=2]', bench.PMC_PROFILE_C5)
    assert t is not None and t['kernel_grid'].endswith('|2162688')  # 352 x 8 blocks x 768
    assert abs(t['write_bytes'] - 89600 * 1024 * 4) < 0.01 * 89600 * 1024 * 4
    assert t['read_bytes_corrected'] > 89600 * 256 * 4  # at least the input once
    assert bench.pmc_traffic_slab('rnn_bidir[gru,B=64,T=200,H=64,mma=2]', bench.PMC_PROFILE_C5) is None
