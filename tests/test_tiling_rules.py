"""Host-side launch rules (CPU): padded LSTM hidden sizes and the GEMM split / tile choices.

The kernels are instantiated for fixed padded per-direction hidden sizes (resident weights up to
192, streamed weights 256 / 384 / 512); a size outside them must report 0 so the model raises
instead of silently running the per-step reference loop.  The grouped weight-gradient GEMM
switches to 128x128 tiles for very long K (large-batch K = B*S) and sizes its split count on
the tile count it actually launches.
"""
from dinunet_implementations_amd.ops import gemm
from dinunet_implementations_amd.ops.lstm import lstm_supported, padded_hidden


def test_padded_hidden_covers_resident_and_streamed_sizes():
    assert [padded_hidden(h) for h in (1, 64, 65, 128, 174, 192)] == [64, 64, 128, 128, 192, 192]
    assert [padded_hidden(h) for h in (193, 256, 300, 384, 385, 512)] == [256, 256, 384, 384, 512, 512]
    assert padded_hidden(513) == 0 and padded_hidden(0) == 0
    assert lstm_supported(32, 256, 512, 2) and not lstm_supported(32, 256, 600, 2)


def test_split_rule_long_k_targets_workgroups_per_cu():
    ncu = gemm._NCU
    k = 2048 * 98  # B = 2048 ICA step: K = B*S
    # ~8 workgroups per CU over the tiles actually launched, capped at 32 and K/2048
    for tiles in (16, 90, 284):
        sp = gemm._split_rule(tiles, k)
        assert 1 <= sp <= 32 and sp * 2048 <= k
        assert sp == min(32, -(-8 * ncu // tiles))
    # 128x128 tile count of the B=2048 grouped launch (~90 tiles) -> 23 splits (measured best 24)
    assert gemm._split_rule(90, k) == min(32, -(-8 * ncu // 90))
    # medium K keeps the old rule; short K never splits
    assert gemm._split_rule(284, 3136) >= 1
    assert gemm._split_rule(284, 256) == 1
    assert gemm._LONG_K == 16384


def test_lstm_backward_rows_tile_the_forward_padding():
    """The backward recurrence may tile the batch with more rows per workgroup than the forward
    (8 vs 4 from B = 2048 at 192 units); its grid must never reach rows past the forward's padded
    buffers, at any batch and hidden size."""
    from dinunet_implementations_amd.ops import _lib
    if not _lib.native_available():
        import pytest
        pytest.skip("kernel library not built")
    L = _lib.lib()
    for hd in (64, 128, 174, 192, 256, 384):
        for B in list(range(1, 70)) + [511, 512, 1023, 1024, 2040, 2044, 2048, 2052, 4096, 4100,
                                       8192, 16384]:
            bf = int(L.dn_lstm_rows_per_wg(B, hd))
            bb = int(L.dn_lstm_rows_per_wg_bwd(B, hd))
            padded = -(-B // bf) * bf
            assert -(-B // bb) * bb <= padded, (hd, B, bf, bb)
    assert int(L.dn_lstm_rows_per_wg(2048, 192)) == 4 and int(L.dn_lstm_rows_per_wg_bwd(2048, 192)) == 8
    assert int(L.dn_lstm_rows_per_wg_bwd(2044, 192)) == 4  # not a multiple of 8: same as forward
    assert int(L.dn_lstm_rows_per_wg_bwd(32, 192)) == 4
