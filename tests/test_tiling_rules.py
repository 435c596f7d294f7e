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
    (8 vs 4 from B = 1024 at 192 units).  It addresses the forward's padded buffers with the
    forward's row count, passed explicitly (``dn_lstm_bwd``'s ``Bp``), so a tiling only has to
    stay inside them: never a row past the forward's padding, at any batch and hidden size."""
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
            # the backward reads the forward's cell states with its own padded batch as the
            # direction stride (lstm.hip bwd_recur): the two paddings must be EQUAL
            assert -(-B // bb) * bb == padded, (hd, B, bf, bb)
    assert int(L.dn_lstm_rows_per_wg(2048, 192)) == 4 and int(L.dn_lstm_rows_per_wg_bwd(2048, 192)) == 8
    assert int(L.dn_lstm_rows_per_wg_bwd(1024, 192)) == 8
    assert int(L.dn_lstm_rows_per_wg_bwd(2044, 192)) == 4  # not a multiple of 8: same as forward
    assert int(L.dn_lstm_rows_per_wg_bwd(32, 192)) == 4


def test_lstm_launchers_refuse_inconsistent_buffers():
    """The host launchers check what the kernels would otherwise read silently wrong, before any
    launch (so this runs without a GPU): a backward given fewer padded rows than the batch, and a
    bf16 pre-activation buffer where the kernels only offer fp32 (the element type
    travels as an explicit argument, not a process-global flag)."""
    import ctypes
    from dinunet_implementations_amd.ops import _lib
    if not _lib.native_available():
        import pytest
        pytest.skip("kernel library not built")
    L = _lib.lib()
    V, I_, Lg, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_long, ctypes.c_float
    L.dn_lstm_bwd.argtypes = [V, V, V, V, Lg, Lg, F, V, V, I_, I_, I_, I_, V, I_, I_, V]
    L.dn_lstm_fwd.argtypes = [V, V, V, I_, I_, I_, I_, V, V, V, V, F, V, V, V, I_, I_, V]
    BAD = 1  # common.h DN_BAD_SHAPE
    # Bp < B
    assert L.dn_lstm_bwd(None, None, None, None, 384, 0, 1.0, None, None, 32, 98, 192, 2, None,
                         16, 0, None) == BAD
    # bf16 pre at 64 units (only the 192-unit resident geometry offers it), and with a sequence
    # output
    assert L.dn_lstm_bwd(None, None, None, None, 128, 0, 1.0, None, None, 32, 98, 64, 2, None,
                         32, 1, None) == BAD
    assert L.dn_lstm_fwd(None, None, None, 32, 98, 64, 2, None, None, None, None, 1.0, None, None,
                         None, 0, 1, None) == BAD
    assert L.dn_lstm_fwd(None, None, None, 32, 98, 192, 2, None, None, ctypes.c_void_p(16),
                         None, 1.0, None, None, None, 0, 1, None) == BAD


def test_tail_rows_cut_only_a_mostly_idle_last_round():
    """ops.gemm._tail_rows: a one-split 256 x 256 launch whose last round would fill at most a
    quarter of the CUs runs those rows as a second launch (r0 = first tail row, a tile boundary);
    full rounds, larger last rounds, split launches and other tiles launch as they are."""
    from dinunet_implementations_amd.ops import gemm
    ncu = gemm._NCU
    M = 2048 * 98                                   # B = 2048 ICA rows: 784 row tiles
    r0 = gemm._tail_rows(M, 256, 1536, 2, 1)
    assert r0 == (784 - 784 % ncu) * 256 and r0 % 256 == 0
    assert gemm._tail_rows(M, 1536, 256, 2, 1) is None      # projection: last round 37.5 % full
    assert gemm._tail_rows(M, 256, 1536, 1, 1) is None      # not the 256 x 256 kernel
    assert gemm._tail_rows(M, 256, 1536, 2, 4) is None      # split-K launches keep their slabs
    assert gemm._tail_rows(256 * ncu * 3, 256, 1536, 2, 1) is None  # whole rounds
    assert gemm._tail_rows(256 * 100, 256, 1536, 2, 1) is None      # one partial round only
    assert gemm._tail_rows(M, 256, 128, 2, 1) is None       # short K: not worth a launch
    old = gemm.GEMM_TAIL
    try:
        gemm.GEMM_TAIL = False
        assert gemm._tail_rows(M, 256, 1536, 2, 1) is None
    finally:
        gemm.GEMM_TAIL = old
