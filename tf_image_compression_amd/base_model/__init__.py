"""Mirror of the reference's base_model/ experiments on the encode/decode path (ch_128)."""
