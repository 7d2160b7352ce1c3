package com.tchaicatkovsky.jleveldb.util;

import java.nio.ByteBuffer;

/**
 * Static natives over libjlcrc.so (include/jlcrc.h) through jlcrc_jni.c.
 * Loaded once; {@link #init(int)} binds the process to its GPU (the reference's
 * Crc32C is static, so there is no per-instance state on the native side).
 */
public final class Crc32CNative {
    static {
        System.loadLibrary("jlcrc_jni");
    }

    private Crc32CNative() {}

    public static native long value(byte[] data, int offset, int n);

    public static native long extend(long initCrc, byte[] data, int offset, int n);

    /** update() on the bit-flipped state held by a Crc32C instance. */
    public static native int update(int state, byte[] data, int offset, int n);

    public static native int init(int device);

    public static native String lastError();

    /** jl_set_option / jl_get_option (include/jlcrc.h JL_OPT_*); 0 or a negative error code. */
    public static native int setOption(int option, long value);

    public static native long getOption(int option);

    /** Host-memory calls touching fewer bytes run on the host's SSE4.2 path (tables, batches). */
    public static final int OPT_HOST_THRESHOLD = 7;
    /** The same for log verification. */
    public static final int OPT_LOG_HOST_THRESHOLD = 8;

    /** TableFormat.readBlock checksum test for many handles of one mmap'd table. */
    public static native int tableVerify(ByteBuffer file, long[] offset, int[] size, byte[] status);

    /**
     * The same for several mmap'd tables at once (a compaction's inputs,
     * VersionSet.makeInputIterator): table t's handles are offset/size[first[t] ..
     * first[t + 1]), first.length == files.length + 1.
     */
    public static native int tablesVerify(ByteBuffer[] files, long[] first, long[] offset, int[] size, byte[] status);

    /**
     * Block handles of a whole mmap'd table (footer, index, metaindex walk):
     * data blocks in index order, meta blocks, metaindex, index.  Returns the
     * handle count (greater than offset.length: grow the arrays and call again)
     * or a negative error code with the Status text in lastError().
     */
    public static native long tableBlockHandles(ByteBuffer file, long[] offset, int[] size, byte[] kind);

    /**
     * LogReader verification of a whole log image; returns the number of 16-byte
     * events (greater than events.capacity() / 16: grow the buffer and call
     * again) or a negative error code.
     */
    public static native long logVerify(ByteBuffer log, boolean checksum, ByteBuffer events);
}
