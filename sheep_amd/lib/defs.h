// Types and constants of the Sheep host API (reference: lib/defs.h:76-82, jnode.h:42-43,
// partition.h:43-44).  The MI355X build keeps the reference's 32-bit id space.
#pragma once
#include <cassert>
#include <cstddef>
#include <cstdint>

typedef uint32_t vid_t;
typedef uint32_t esize_t;
typedef vid_t jnid_t;
typedef short part_t;

#define INVALID_VID ((vid_t)-1)
#define INVALID_JNID ((jnid_t)-1)
#define INVALID_PART ((part_t)-1)

#define KILO (1024)
#define MEGA (1024 * KILO)
#define GIGA (1024 * MEGA)
