package vproxy.component.secure;

import vproxybase.util.Utils;

/**
 * Selects the classifier implementation, the way vfd/VFDConfig.java:27-41
 * selects the fd implementation:
 *
 * <pre>
 *   -Dclassifier=gpu            use libvclassify for the batched drain loops
 *                               (default: java, the reference's scans)
 *   -Dclassifier_lib=NAME       JNI library name (default vclassify_jni)
 *   -Dclassifier_device=N       GPU ordinal (default 0)
 *   -Dclassifier_batch=N        most datagrams per drain-loop batch (default 4096)
 * </pre>
 *
 * With the default nothing here loads a native library and every caller
 * keeps the reference code path unchanged.
 */
public class ClassifierConfig {
    private ClassifierConfig() {
    }

    public static final String classifierImpl;
    public static final boolean useGpu;
    public static final String libname;
    public static final int device;
    public static final int batch;

    static {
        classifierImpl = Utils.getSystemProperty("classifier", "java");
        useGpu = classifierImpl.equals("gpu");
        libname = Utils.getSystemProperty("classifier_lib", "vclassify_jni");
        device = Integer.parseInt(Utils.getSystemProperty("classifier_device", "0"));
        int b = Integer.parseInt(Utils.getSystemProperty("classifier_batch", "4096"));
        batch = b < 1 ? 1 : b;
    }
}
