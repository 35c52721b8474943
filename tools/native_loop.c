/* native_loop.c — bench helper, not part of the library: the reference's
 * criterion loop (benches/performance_microbenchmarks.rs:43-64,
 * b.iter(|| fill_controlled_data(&mut buf, dedup, compress))) as a native
 * caller of the C ABI, so bench.py configs 11-13 time the calls the way a
 * Rust caller makes them, without Python's ~2 us per ctypes call.  The entry
 * point is passed in (the library's own s3dg_fill_controlled), so this file
 * links against nothing. */
#include <stdint.h>

typedef int (*fill_fn)(void *ctx, void *dst, uint64_t len, uint64_t dedup, uint32_t f_num, uint32_t f_den,
                       uint64_t entropy, void *stream);

__attribute__((visibility("default"))) int nl_fill_loop(void *fn, void *ctx, void *dst, uint64_t len,
                                                        uint64_t calls, uint64_t dedup, uint32_t f_num,
                                                        uint32_t f_den, uint64_t entropy, void *stream) {
    const fill_fn f = (fill_fn)fn;
    for (uint64_t k = 0; k < calls; ++k) {
        const int r = f(ctx, dst, len, dedup, f_num, f_den, entropy, stream);
        if (r) return r;
    }
    return 0;
}
