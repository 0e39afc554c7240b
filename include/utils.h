/* utils.h — drop-in for ray-tracing-c include/utils.h (reference include/utils.h:1-33).
 *
 * Constants and helper macros that reference-style drivers (main.c) rely on.  clamp() keeps the
 * reference's ternary semantics (a NaN input clamps to `lo`), which the quantizer in
 * Camera_render depends on (reference src/raytracing.c:129).
 */
#ifndef RT_UTILS_H
#define RT_UTILS_H
#ifndef UTILS_H
#define UTILS_H
#endif

#include <assert.h>
#include <stdlib.h>

/* -std=c11 does not provide these */
#ifndef M_PI
#define M_PI 3.14159265358979323846264338327950288
#endif
#ifndef M_1_PI
#define M_1_PI 0.318309886183790671537767526745028724
#endif

#ifndef min
#define min(a, b) ((a) < (b) ? (a) : (b))
#endif
#ifndef max
#define max(a, b) ((a) > (b) ? (a) : (b))
#endif
#define clamp(v, lo, hi) min(max(v, lo), hi)

/* heap-allocate a Type and brace-initialise it (reference include/utils.h:19-24) */
#define define_struct_new(Type, ...)                                                                \
  {                                                                                                \
    Type *obj_ = my_malloc(sizeof(Type));                                                          \
    *obj_ = (Type){__VA_ARGS__};                                                                   \
    return obj_;                                                                                   \
  }
/* heap-allocate a Type and run Type_init on it (reference include/utils.h:25-30) */
#define define_init_new(Type, ...)                                                                 \
  {                                                                                                \
    Type *obj_ = my_malloc(sizeof(Type));                                                          \
    Type##_init(obj_, ##__VA_ARGS__);                                                              \
    return (void *)obj_;                                                                           \
  }

/* malloc that aborts on failure (reference src/utils.c:3-7) */
void *my_malloc(size_t size);

#endif /* RT_UTILS_H */
