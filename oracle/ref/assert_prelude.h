/* Force-included ahead of every reference source this directory compiles
 * (Makefile, -include).  TEST INFRASTRUCTURE ONLY.
 *
 * common/misc/log.h is the one reference header that reads NDEBUG
 * (log.h:80-137): without it, LOG_* call a logging back end (log.cc) that
 * needs Boost, which this image lacks.  So log.h is read once with NDEBUG
 * defined (its include guard keeps that choice), then NDEBUG is dropped and
 * <assert.h> re-read: the reference's own assert() calls stay active in the
 * controllers, caches and queue models the fixtures come from.  Nothing of
 * the reference is replaced; no other reference file reads NDEBUG. */
#ifndef GG_ASSERT_PRELUDE_H
#define GG_ASSERT_PRELUDE_H
#define NDEBUG
#include "log.h"
#undef NDEBUG
#include <assert.h>
#endif
